// cn_fields.hip — per-row encodings around the MLP GEMMs (gfx950).
//
// All kernels use one thread per (row, float4 column group): 16 consecutive
// threads cover one 64-float row, so loads and stores are fully coalesced
// 16-byte accesses.  Layout of the SDF encoding (neus_embedder.py:17-36,
// include_input, log bands, periodic_fns [sin, cos], d = 4):
//   group 0        : x' = scale * x                      (cols 0..3)
//   group 1 + 2k   : sin(2^k x')                         (k < multires)
//   group 2 + 2k   : cos(2^k x')
//   groups >= 1+2L : zero padding up to kpad
#include "cn_common.h"

namespace cn {

__device__ __forceinline__ floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }
__device__ __forceinline__ void st4(float* p, floatx4 v) { *reinterpret_cast<floatx4*>(p) = v; }
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
// 4 values into row m, columns 4g.. of a tail buffer: fp32, or (bf16) the RNE bf16 operand image
__device__ __forceinline__ void st4_tail(void* base, bool bf16, int64_t m, int64_t ld, int g, floatx4 v) {
    if (bf16)
        *reinterpret_cast<bf16x4_t*>(static_cast<__bf16*>(base) + m * ld + 4 * g) = __builtin_convertvector(v, bf16x4_t);
    else
        st4(static_cast<float*>(base) + m * ld + 4 * g, v);
}

__global__ void sdf_embed_kernel(int M, const float* __restrict__ x, int64_t ldx, int L, float scale, int G,
                                 void* U0, int64_t ld_u0, bool u0b, void* U4e, int64_t ld_u4, float u4div, bool u4b) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = idx / G;
    const int g = idx % G;
    if (m >= M) return;
    const floatx4 o = sdf_embed_group(ld4(x + m * ldx), g, L, scale);
    const int ng = 1 + 2 * L;
    st4_tail(U0, u0b, m, ld_u0, g, o);
    if (U4e && g < ng) {
        floatx4 q;
        for (int c = 0; c < 4; ++c) q[c] = o[c] / u4div;
        st4_tail(U4e, u4b, m, ld_u4, g, q);
    }
}

// G[m] = scale * sum_groups J_groupᵀ (Q0 + QE)[group].  16 (or 8) lanes per row
// reduce with xor shuffles inside their group of G lanes.
__global__ void sdf_grad_assemble_kernel(int M, int L, float scale, int G, const float* __restrict__ U0,
                                         int64_t ld_u0, const float* __restrict__ Q0, int64_t ld_q0,
                                         const float* __restrict__ QE, int64_t ld_qe, float* out, int64_t ld_g) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = idx / G;
    const int g = idx % G;
    const bool valid = m < M;
    const int ng = 1 + 2 * L;
    floatx4 c = {0.f, 0.f, 0.f, 0.f};
    if (valid && g < ng) {
        floatx4 de = ld4(Q0 + m * ld_q0 + 4 * g);
        if (QE) {
            const floatx4 e = ld4(QE + m * ld_qe + 4 * g);
            for (int q = 0; q < 4; ++q) de[q] = de[q] + e[q];
        }
        if (g == 0) {
            c = de;
        } else {
            const int k = (g - 1) >> 1;
            const float f = (float)(1 << k);
            const bool is_sin = ((g - 1) & 1) == 0;
            // d sin(t)/dt = cos(t) (stored in the next group), d cos(t)/dt = -sin(t)
            const floatx4 tr = ld4(U0 + m * ld_u0 + 4 * (is_sin ? g + 1 : g - 1));
            for (int q = 0; q < 4; ++q) c[q] = (is_sin ? de[q] * tr[q] : de[q] * (-tr[q])) * f;
        }
    }
    for (int off = G >> 1; off > 0; off >>= 1)
        for (int q = 0; q < 4; ++q) c[q] += __shfl_xor(c[q], off, G);
    if (valid && g == 0) {
        floatx4 o;
        for (int q = 0; q < 4; ++q) o[q] = c[q] * scale;
        st4(out + m * ld_g, o);
    }
}

// T0[m][group] = J_group(x') * (scale * v[m]); the forward-mode tangent of the
// encoding along v = dL/d(gradient) (double backward of neus_fields.py:296).
__global__ void sdf_tangent_prep_kernel(int M, int L, float scale, int G, const float* __restrict__ U0,
                                        int64_t ld_u0, const float* __restrict__ v, int64_t ld_v, float* T0,
                                        int64_t ld_t0, void* T4e, int64_t ld_t4, float t4div, bool t4b) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = idx / G;
    const int g = idx % G;
    if (m >= M) return;
    const int ng = 1 + 2 * L;
    floatx4 o = {0.f, 0.f, 0.f, 0.f};
    if (g < ng) {
        const floatx4 vv = ld4(v + m * ld_v);
        floatx4 xd;
        for (int q = 0; q < 4; ++q) xd[q] = vv[q] * scale;
        if (g == 0) {
            o = xd;
        } else {
            const int k = (g - 1) >> 1;
            const float f = (float)(1 << k);
            const bool is_sin = ((g - 1) & 1) == 0;
            const floatx4 tr = ld4(U0 + m * ld_u0 + 4 * (is_sin ? g + 1 : g - 1));
            for (int q = 0; q < 4; ++q) {
                const float td = xd[q] * f;
                o[q] = is_sin ? tr[q] * td : (-tr[q]) * td;
            }
        }
    }
    st4(T0 + m * ld_t0 + 4 * g, o);
    if (T4e && g < ng) {
        floatx4 q4;
        for (int q = 0; q < 4; ++q) q4[q] = o[q] / t4div;
        st4_tail(T4e, t4b, m, ld_t4, g, q4);
    }
}

// Colour-network extras, rows [g(4) | pts_time(4) | embed_view(dirs) (3+6L) | 0...]: the view encoding (sin / cos of the ray direction at
// 2^k) is computed once per ray into LDS, not once per sample (dir_div samples share a ray),
// then every row is a copy.  kExtRows rows per workgroup, so at most kExtRows / dir_div + 2 rays.
constexpr int kExtRows = 64;
__global__ void __launch_bounds__(256) color_extras_kernel(int M, const float* __restrict__ Gm, int64_t ld_g,
                                                           const float* __restrict__ pts, int64_t ld_p,
                                                           const float* __restrict__ dirs, int64_t ld_d, int dir_div,
                                                           int L, int G, float* ext, int64_t ld_ext) {
    __shared__ __attribute__((aligned(16))) float emb[kExtRows + 1][32];
    const int64_t m0 = (int64_t)blockIdx.x * kExtRows;
    const int64_t r0 = m0 / dir_div;
    const int64_t mlast = min((int64_t)M, m0 + kExtRows) - 1;
    const int nr = (int)(mlast / dir_div - r0) + 1;
    const int nv = 3 + 6 * L;
    for (int i = threadIdx.x; i < nr * 32; i += blockDim.x) {
        const int rr = i >> 5, e = i & 31;
        float v = 0.f;
        if (e < nv) {
            const float* d = dirs + (r0 + rr) * ld_d;
            if (e < 3) {
                v = d[e];
            } else {
                const int j = e - 3;
                const int k = j / 6, w = j % 6;
                const float t = d[w % 3] * (float)(1 << k);
                v = (w < 3) ? sinf(t) : cosf(t);
            }
        }
        emb[rr][e] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kExtRows * G; i += blockDim.x) {
        const int64_t m = m0 + i / G;
        const int g = i % G;
        if (m >= M) break;  // rows grow with i
        floatx4 o = {0.f, 0.f, 0.f, 0.f};
        if (g == 0) {
            o = ld4(Gm + m * ld_g);
        } else if (g == 1) {
            o = ld4(pts + m * ld_p);
        } else if (4 * (g - 2) < 32) {
            o = *reinterpret_cast<const floatx4*>(&emb[m / dir_div - r0][4 * (g - 2)]);
        }
        st4(ext + m * ld_ext + 4 * g, o);
    }
}

// Gradient of the per-ray view directions through the view encoding.  Block =
// 8 rays x 32 lanes; lane e < nv sums column 8+e of d_ext over the ray's rows
// (double, fixed order), then lanes 0..2 apply the encoding's Jacobian.
__global__ void __launch_bounds__(256) color_extras_bwd_kernel(int R, int rows, const float* __restrict__ d_ext,
                                                               int64_t ld_ext, const float* __restrict__ dirs,
                                                               int64_t ld_d, int L, float* ddirs, int accumulate) {
    __shared__ double part[8][32];
    const int rr = threadIdx.x >> 5, e = threadIdx.x & 31;
    const int r = blockIdx.x * 8 + rr;
    const int nv = 3 + 6 * L;
    double acc = 0.0;
    if (r < R && e < nv) {
        const float* col = d_ext + (int64_t)r * rows * ld_ext + 8 + e;
        for (int i = 0; i < rows; ++i) acc += (double)col[(int64_t)i * ld_ext];
    }
    part[rr][e] = acc;
    __syncthreads();
    if (r < R && e < 3) {
        const float dc = dirs[(int64_t)r * ld_d + e];
        double g = part[rr][e];
        for (int k = 0; k < L; ++k) {
            const float f = (float)(1 << k);
            const float t = dc * f;
            // ext column 3 + 6k + w: w < 3 sin(2^k d_w), w >= 3 cos(2^k d_{w-3})
            g += (double)(f * cosf(t)) * part[rr][3 + 6 * k + e] - (double)(f * sinf(t)) * part[rr][3 + 6 * k + 3 + e];
        }
        float* o = ddirs + 3 * (int64_t)r + e;
        *o = accumulate ? *o + (float)g : (float)g;
    }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace cn

using namespace cn;

extern "C" int cn_sdf_embed(int32_t M, const float* x, int64_t ldx, int32_t multires, float scale, int32_t kpad,
                            void* U0, int64_t ld_u0, void* U4e, int64_t ld_u4, float u4_scale, int32_t flags,
                            cn_stream_t stream) {
    CN_REQUIRE(x && U0, CN_ERR_ARG, "cn_sdf_embed: null pointer");
    CN_REQUIRE(multires >= 0 && 4 * (1 + 2 * multires) <= kpad && kpad % 4 == 0 && ld_u0 >= kpad && multires < 16,
               CN_ERR_SHAPE, "cn_sdf_embed: multires=%d kpad=%d ld_u0=%lld", multires, kpad, (long long)ld_u0);
    const bool u0b = (flags & 2) != 0;
    CN_REQUIRE(al16(x) && ((uintptr_t)U0 & (u0b ? 7 : 15)) == 0 && ldx % 4 == 0 && ld_u0 % 4 == 0 &&
                   (!U4e || (((uintptr_t)U4e & 7) == 0 && ld_u4 % 4 == 0)),
               CN_ERR_ALIGN, "cn_sdf_embed: alignment");
    if (M == 0) return CN_OK;
    const int G = kpad / 4;
    const int64_t tot = (int64_t)M * G;
    sdf_embed_kernel<<<(int)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        M, x, ldx, multires, scale, G, U0, ld_u0, u0b, U4e, ld_u4, u4_scale == 0.f ? 1.f : u4_scale, (flags & 1) != 0);
    return check_launch("cn_sdf_embed");
}

extern "C" int cn_sdf_grad_assemble(int32_t M, int32_t multires, float scale, const float* U0, int64_t ld_u0,
                                    const float* Q0, int64_t ld_q0, const float* QE, int64_t ld_qe, float* G,
                                    int64_t ld_g, cn_stream_t stream) {
    CN_REQUIRE(U0 && Q0 && G, CN_ERR_ARG, "cn_sdf_grad_assemble: null pointer");
    const int ng = 1 + 2 * multires;
    const int Gl = ng <= 8 ? 8 : 16;
    CN_REQUIRE(ng <= 16, CN_ERR_UNSUPPORTED, "cn_sdf_grad_assemble: multires=%d", multires);
    CN_REQUIRE(al16(U0) && al16(Q0) && al16(G) && (!QE || al16(QE)) && ld_u0 % 4 == 0 && ld_q0 % 4 == 0 &&
                   ld_g % 4 == 0 && ld_qe % 4 == 0,
               CN_ERR_ALIGN, "cn_sdf_grad_assemble: alignment");
    if (M == 0) return CN_OK;
    const int64_t tot = (int64_t)M * Gl;
    sdf_grad_assemble_kernel<<<(int)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        M, multires, scale, Gl, U0, ld_u0, Q0, ld_q0, QE, ld_qe, G, ld_g);
    return check_launch("cn_sdf_grad_assemble");
}

extern "C" int cn_sdf_tangent_prep(int32_t M, int32_t multires, float scale, int32_t kpad, const float* U0,
                                   int64_t ld_u0, const float* v, int64_t ld_v, float* T0, int64_t ld_t0, void* T4e,
                                   int64_t ld_t4, float t4_scale, int32_t t4_bf16, cn_stream_t stream) {
    CN_REQUIRE(U0 && v && T0, CN_ERR_ARG, "cn_sdf_tangent_prep: null pointer");
    CN_REQUIRE(4 * (1 + 2 * multires) <= kpad && kpad % 4 == 0 && ld_t0 >= kpad, CN_ERR_SHAPE,
               "cn_sdf_tangent_prep: kpad");
    CN_REQUIRE(al16(U0) && al16(v) && al16(T0) && (!T4e || (((uintptr_t)T4e & 7) == 0 && ld_t4 % 4 == 0)) &&
                   ld_v % 4 == 0 && ld_t0 % 4 == 0,
               CN_ERR_ALIGN, "cn_sdf_tangent_prep: alignment");
    if (M == 0) return CN_OK;
    const int G = kpad / 4;
    const int64_t tot = (int64_t)M * G;
    sdf_tangent_prep_kernel<<<(int)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        M, multires, scale, G, U0, ld_u0, v, ld_v, T0, ld_t0, T4e, ld_t4, t4_scale == 0.f ? 1.f : t4_scale,
        t4_bf16 != 0);
    return check_launch("cn_sdf_tangent_prep");
}

extern "C" int cn_color_extras(int32_t M, const float* G, int64_t ld_g, const float* pts, int64_t ld_p,
                               const float* dirs, int64_t ld_d, int32_t dir_div, int32_t multires_view, int32_t kpad,
                               float* ext, int64_t ld_ext, cn_stream_t stream) {
    CN_REQUIRE(G && pts && dirs && ext, CN_ERR_ARG, "cn_color_extras: null pointer");
    CN_REQUIRE(dir_div >= 1, CN_ERR_ARG, "cn_color_extras: dir_div");
    CN_REQUIRE(8 + 3 + 6 * multires_view <= kpad && kpad % 4 == 0 && ld_ext >= kpad, CN_ERR_SHAPE,
               "cn_color_extras: kpad=%d too small for multires_view=%d", kpad, multires_view);
    CN_REQUIRE(al16(G) && al16(pts) && al16(ext) && ld_g % 4 == 0 && ld_p % 4 == 0 && ld_ext % 4 == 0,
               CN_ERR_ALIGN, "cn_color_extras: alignment");
    CN_REQUIRE(3 + 6 * multires_view <= 32, CN_ERR_UNSUPPORTED, "cn_color_extras: multires_view=%d", multires_view);
    if (M == 0) return CN_OK;
    const int Gc = kpad / 4;
    color_extras_kernel<<<cdiv(M, kExtRows), 256, 0, (hipStream_t)stream>>>(
        M, G, ld_g, pts, ld_p, dirs, ld_d, dir_div, multires_view, Gc, ext, ld_ext);
    return check_launch("cn_color_extras");
}

extern "C" int cn_color_extras_bwd(int32_t R, int32_t dir_div, const float* d_ext, int64_t ld_ext, const float* dirs,
                                   int64_t ld_d, int32_t multires_view, float* ddirs, int32_t accumulate,
                                   cn_stream_t stream) {
    CN_REQUIRE(d_ext && dirs && ddirs, CN_ERR_ARG, "cn_color_extras_bwd: null pointer");
    CN_REQUIRE(R >= 0 && dir_div >= 1 && multires_view >= 0 && 3 + 6 * multires_view <= 32 &&
                   ld_ext >= 8 + 3 + 6 * multires_view && ld_d >= 3,
               CN_ERR_SHAPE, "cn_color_extras_bwd: R=%d dir_div=%d multires_view=%d", R, dir_div, multires_view);
    if (R == 0) return CN_OK;
    color_extras_bwd_kernel<<<cdiv(R, 8), 256, 0, (hipStream_t)stream>>>(R, dir_div, d_ext, ld_ext, dirs, ld_d,
                                                                        multires_view, ddirs, accumulate);
    return check_launch("cn_color_extras_bwd");
}
