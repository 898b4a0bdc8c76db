// cn_stage1.hip — the per-sample work of the stage-1 losses (train.py:467-505) in one
// pass over the samples each way, instead of ~40 torch launches (several of them
// full-length reductions torch runs with a handful of threads):
//
//   scene-flow SDF loss (train.py:470-477)  e_m = (ω × p_m + v) · n_m + f_m,
//                                           num = Σ_m |e_m| w_m, Σ_m w_m (w detached);
//   flow projection (train.py:484-495)      per ray r: Σ_s w p, Σ_s w (the reference maps
//                                           every sample and averages; by linearity the
//                                           per-ray sums carry the whole projection);
//   SDF-consistency points (train.py:502-504)  x_m = [cw2 (p_m, 1), t_world].
//
// One wavefront per ray (lanes stride over its samples), four rays per workgroup;
// the two global sums and, backward, the ω / v / cw2 gradients are per-workgroup
// partials summed in a fixed order (slab_reduce_kernel): bitwise reproducible.
#include "cn_mfma.h"

namespace cn {

struct Stage1Ptrs {
    const float* pts;      // [M] rows of >= 3 (ld_p)
    const float* nrm;      // [M] rows of >= 3 (ld_n): ∇ₓ sdf
    const float* flw;      // [M] (stride ld_f): ∂sdf/∂t
    const float* w;        // [R, S] render weights
    const float* mv;       // [6]: ω, v
    const float* cw2;      // [4, 4] or null
    int ld_p, ld_n, ld_f;
};

__device__ __forceinline__ float3 ld3(const float* p) { return make_float3(p[0], p[1], p[2]); }
__device__ __forceinline__ float3 cross3(float3 a, float3 b) {
    return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float dot3(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

template <int N>
__device__ __forceinline__ void wave_sum(float (&v)[N]) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] += __shfl_xor(v[i], o, 64);
}

// Workgroup partials of N sums in a fixed order: wave sums, then waves 0..3 in order.
template <int N>
__device__ __forceinline__ void block_partials(float (&v)[N], float* smem, float* part) {
    wave_sum<N>(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < N; ++i) smem[wave * N + i] = v[i];
    __syncthreads();
    if (threadIdx.x < N) {
        const int i = threadIdx.x;
        part[(int64_t)blockIdx.x * N + i] = ((smem[i] + smem[N + i]) + smem[2 * N + i]) + smem[3 * N + i];
    }
}

__global__ void __launch_bounds__(256) stage1_fwd_kernel(int R, int S, Stage1Ptrs a, float t_world, float* ray_acc,
                                                         float* x_out, int64_t ld_x, float* part) {
    __shared__ float smem[4 * 2];
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const float3 om = make_float3(a.mv[0], a.mv[1], a.mv[2]);
    const float3 vel = make_float3(a.mv[3], a.mv[4], a.mv[5]);
    float c[12] = {};
    if (a.cw2)
#pragma unroll
        for (int i = 0; i < 12; ++i) c[i] = a.cw2[i];
    float sums[2] = {0.f, 0.f};  // Σ |e| w, Σ w
    float racc[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < R) {
        for (int s = lane; s < S; s += 64) {
            const int64_t m = (int64_t)r * S + s;
            const float3 p = ld3(a.pts + m * a.ld_p);
            const float3 n = ld3(a.nrm + m * a.ld_n);
            const float f = a.flw[m * a.ld_f];
            const float w = a.w[m];
            const float3 fl = cross3(om, p);
            const float e = ((fl.x + vel.x) * n.x + (fl.y + vel.y) * n.y + (fl.z + vel.z) * n.z) + f;
            sums[0] += fabsf(e) * w;
            sums[1] += w;
            racc[0] += w * p.x;
            racc[1] += w * p.y;
            racc[2] += w * p.z;
            racc[3] += w;
            if (x_out) {
                float* x = x_out + m * ld_x;
                x[0] = c[0] * p.x + c[1] * p.y + c[2] * p.z + c[3];
                x[1] = c[4] * p.x + c[5] * p.y + c[6] * p.z + c[7];
                x[2] = c[8] * p.x + c[9] * p.y + c[10] * p.z + c[11];
                x[3] = t_world;
            }
        }
    }
    wave_sum<4>(racc);
    if (r < R && lane == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) ray_acc[(int64_t)r * 4 + i] = racc[i];
    block_partials<2>(sums, smem, part);
}

// g_num: dL/d(Σ|e| w) (device scalar); d_ray [R, 4] and dx [M] rows (ld_dx) optional.
__global__ void __launch_bounds__(256) stage1_bwd_kernel(int R, int S, Stage1Ptrs a, const float* g_num,
                                                         const float* d_ray, const float* dx, int64_t ld_dx,
                                                         float* dnrm, int64_t ld_dn, float* dflw, int64_t ld_df,
                                                         float* dw, float* dpts, int64_t ld_dp, float* part) {
    __shared__ float smem[4 * 18];
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const float3 om = make_float3(a.mv[0], a.mv[1], a.mv[2]);
    const float3 vel = make_float3(a.mv[3], a.mv[4], a.mv[5]);
    float c[9] = {};
    if (a.cw2)
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) c[i * 3 + j] = a.cw2[i * 4 + j];
    const float g = g_num ? g_num[0] : 0.0f;
    float acc[18] = {};  // dω (3), dv (3), dcw2 rows 0..2 (4 each)
    if (r < R) {
        float4 dr = make_float4(0.f, 0.f, 0.f, 0.f);
        if (d_ray) dr = *reinterpret_cast<const float4*>(d_ray + (int64_t)r * 4);
        for (int s = lane; s < S; s += 64) {
            const int64_t m = (int64_t)r * S + s;
            const float3 p = ld3(a.pts + m * a.ld_p);
            const float3 n = ld3(a.nrm + m * a.ld_n);
            const float f = a.flw[m * a.ld_f];
            const float w = a.w[m];
            const float3 fl0 = cross3(om, p);
            const float3 fl = make_float3(fl0.x + vel.x, fl0.y + vel.y, fl0.z + vel.z);
            const float e = dot3(fl, n) + f;
            const float sg = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);  // torch.abs backward: sgn, 0 at 0
            const float q = g * w * sg;
            float* o = dnrm + m * ld_dn;
            o[0] = q * fl.x;
            o[1] = q * fl.y;
            o[2] = q * fl.z;
            dflw[m * ld_df] = q;
            const float3 pn = cross3(p, n);
            acc[0] += q * pn.x;
            acc[1] += q * pn.y;
            acc[2] += q * pn.z;
            acc[3] += q * n.x;
            acc[4] += q * n.y;
            acc[5] += q * n.z;
            float3 gp = make_float3(0.f, 0.f, 0.f);
            if (dpts) {  // (ω × p) · n = p · (n × ω)
                const float3 nw = cross3(n, om);
                gp = make_float3(q * nw.x + w * dr.x, q * nw.y + w * dr.y, q * nw.z + w * dr.z);
            }
            if (dw) dw[m] = (dr.x * p.x + dr.y * p.y + dr.z * p.z) + dr.w;
            if (dx) {
                const float* d = dx + m * ld_dx;
                const float d0 = d[0], d1 = d[1], d2 = d[2];
                acc[6] += d0 * p.x; acc[7] += d0 * p.y; acc[8] += d0 * p.z; acc[9] += d0;
                acc[10] += d1 * p.x; acc[11] += d1 * p.y; acc[12] += d1 * p.z; acc[13] += d1;
                acc[14] += d2 * p.x; acc[15] += d2 * p.y; acc[16] += d2 * p.z; acc[17] += d2;
                if (dpts) {  // x = cw2[:3, :3] p + cw2[:3, 3]
                    gp.x += c[0] * d0 + c[3] * d1 + c[6] * d2;
                    gp.y += c[1] * d0 + c[4] * d1 + c[7] * d2;
                    gp.z += c[2] * d0 + c[5] * d1 + c[8] * d2;
                }
            }
            if (dpts) {
                float* dp = dpts + m * ld_dp;
                dp[0] = gp.x;
                dp[1] = gp.y;
                dp[2] = gp.z;
            }
        }
    }
    block_partials<18>(acc, smem, part);
}

// Running products of 4x4 matrices, C_0 = A_0, C_j = A_j C_{j-1} (the relative-pose chains of
// stage 1: compute_w2c_mappings, neus_fields.py:171-183, and the masked world-camera chain),
// and their adjoint: G_j = dC_j + A_{j+1}^T G_{j+1}, dA_j = G_j C_{j-1}^T (C_{-1} = I).  A
// chain is a few dozen 4x4 steps: one lane walks it (sequential by nature), instead of a
// rocBLAS launch per product each way.
__device__ __forceinline__ void mm4(const float* a, const float* b, float* c) {  // c = a b
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            c[r * 4 + q] = ((a[r * 4] * b[q] + a[r * 4 + 1] * b[4 + q]) + a[r * 4 + 2] * b[8 + q]) + a[r * 4 + 3] * b[12 + q];
}

__global__ void mat4_chain_fwd_kernel(int n, const float* __restrict__ A, float* C) {
    if (threadIdx.x != 0) return;
    float cur[16], nxt[16], a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) cur[i] = A[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) C[i] = cur[i];
    for (int j = 1; j < n; ++j) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = A[j * 16 + i];
        mm4(a, cur, nxt);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            cur[i] = nxt[i];
            C[j * 16 + i] = nxt[i];
        }
    }
}

__global__ void mat4_chain_bwd_kernel(int n, const float* __restrict__ A, const float* __restrict__ C,
                                      const float* __restrict__ dC, float* dA) {
    if (threadIdx.x != 0) return;
    float G[16], t[16], at[16], ct[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) G[i] = 0.0f;
    for (int j = n - 1; j >= 0; --j) {
        if (j + 1 < n) {  // G <- A_{j+1}^T G
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) at[r * 4 + q] = A[(j + 1) * 16 + q * 4 + r];
            mm4(at, G, t);
#pragma unroll
            for (int i = 0; i < 16; ++i) G[i] = t[i];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) G[i] += dC[j * 16 + i];
        if (j == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) dA[i] = G[i];
        } else {  // dA_j = G C_{j-1}^T
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) ct[r * 4 + q] = C[(j - 1) * 16 + q * 4 + r];
            mm4(G, ct, t);
#pragma unroll
            for (int i = 0; i < 16; ++i) dA[j * 16 + i] = t[i];
        }
    }
}

}  // namespace cn

using namespace cn;

extern "C" size_t cn_stage1_workspace_bytes(int32_t R) {
    const int nblk = cdiv(std::max(R, 1), 4);
    return sizeof(float) * (size_t)nblk * 18;
}

static int stage1_check(int R, int S, const Stage1Ptrs& a, const char* who) {
    CN_REQUIRE(R >= 0 && S > 0, CN_ERR_SHAPE, "%s: bad R=%d S=%d", who, R, S);
    CN_REQUIRE(R == 0 || (a.pts && a.nrm && a.flw && a.w && a.mv), CN_ERR_ARG, "%s: pts, normals, flows, weights, mv required", who);
    CN_REQUIRE(a.ld_p >= 3 && a.ld_n >= 3 && a.ld_f >= 1, CN_ERR_SHAPE, "%s: bad leading dimensions", who);
    return CN_OK;
}

extern "C" int cn_stage1_fwd(int32_t R, int32_t S, const float* pts, int64_t ld_p, const float* normals, int64_t ld_n,
                             const float* flows, int64_t ld_f, const float* weights, const float* mv, const float* cw2,
                             float t_world, float* ray_acc, float* x_out, int64_t ld_x, float* sums,
                             float* workspace, cn_stream_t stream) {
    Stage1Ptrs a{pts, normals, flows, weights, mv, cw2, (int)ld_p, (int)ld_n, (int)ld_f};
    if (int rc = stage1_check(R, S, a, "cn_stage1_fwd")) return rc;
    CN_REQUIRE((R == 0 || ray_acc) && sums && workspace && al16(ray_acc), CN_ERR_ARG,
               "cn_stage1_fwd: ray_acc (16B aligned), sums and workspace required");
    CN_REQUIRE(!x_out || (cw2 && ld_x >= 4), CN_ERR_ARG, "cn_stage1_fwd: x_out needs cw2 and ld_x >= 4");
    hipStream_t s = (hipStream_t)stream;
    const int nblk = cdiv(R, 4);  // R = 0: no samples, the reduction writes zero sums
    if (R > 0) stage1_fwd_kernel<<<nblk, 256, 0, s>>>(R, S, a, t_world, ray_acc, x_out, ld_x, workspace);
    int rc = check_launch("cn_stage1_fwd");
    return rc ? rc : launch_slab_reduce(workspace, nblk, 2, 1, 2, 2, sums, 2, 1.0f, 0, s);
}

extern "C" int cn_stage1_bwd(int32_t R, int32_t S, const float* pts, int64_t ld_p, const float* normals, int64_t ld_n,
                             const float* flows, int64_t ld_f, const float* weights, const float* mv, const float* cw2,
                             const float* g_num, const float* d_ray, const float* dx, int64_t ld_dx, float* dnormals,
                             int64_t ld_dn, float* dflows, int64_t ld_df, float* dweights, float* dpts, int64_t ld_dp,
                             float* dmv_dcw2, float* workspace, cn_stream_t stream) {
    Stage1Ptrs a{pts, normals, flows, weights, mv, cw2, (int)ld_p, (int)ld_n, (int)ld_f};
    if (int rc = stage1_check(R, S, a, "cn_stage1_bwd")) return rc;
    CN_REQUIRE(g_num && (R == 0 || (dnormals && dflows)) && dmv_dcw2 && workspace, CN_ERR_ARG,
               "cn_stage1_bwd: g_num, dnormals, dflows, dmv_dcw2 and workspace required");
    CN_REQUIRE(!dx || (cw2 && ld_dx >= 3), CN_ERR_ARG, "cn_stage1_bwd: dx needs cw2 and ld_dx >= 3");
    CN_REQUIRE(!d_ray || al16(d_ray), CN_ERR_ALIGN, "cn_stage1_bwd: d_ray must be 16B aligned");
    CN_REQUIRE(ld_dn >= 3 && ld_df >= 1 && (!dpts || ld_dp >= 3), CN_ERR_SHAPE, "cn_stage1_bwd: bad output strides");
    hipStream_t s = (hipStream_t)stream;
    const int nblk = cdiv(R, 4);
    if (R > 0)
        stage1_bwd_kernel<<<nblk, 256, 0, s>>>(R, S, a, g_num, d_ray, dx, ld_dx, dnormals, ld_dn, dflows, ld_df, dweights,
                                           dpts, ld_dp, workspace);
    int rc = check_launch("cn_stage1_bwd");
    return rc ? rc : launch_slab_reduce(workspace, nblk, 18, 1, 18, 18, dmv_dcw2, 18, 1.0f, 0, s);
}

extern "C" int cn_mat4_chain_fwd(int32_t n, const float* A, float* C, cn_stream_t stream) {
    CN_REQUIRE(n >= 0 && (n == 0 || (A && C)), CN_ERR_ARG, "cn_mat4_chain_fwd: n=%d, A and C required", n);
    if (n == 0) return CN_OK;
    mat4_chain_fwd_kernel<<<1, 64, 0, (hipStream_t)stream>>>(n, A, C);
    return check_launch("cn_mat4_chain_fwd");
}

extern "C" int cn_mat4_chain_bwd(int32_t n, const float* A, const float* C, const float* dC, float* dA,
                                 cn_stream_t stream) {
    CN_REQUIRE(n >= 0 && (n == 0 || (A && C && dC && dA)), CN_ERR_ARG,
               "cn_mat4_chain_bwd: n=%d, A, C, dC and dA required", n);
    if (n == 0) return CN_OK;
    mat4_chain_bwd_kernel<<<1, 64, 0, (hipStream_t)stream>>>(n, A, C, dC, dA);
    return check_launch("cn_mat4_chain_bwd");
}
