// cn_loss.hip — the training losses of the hot path (gfx950): the loss value and
// its input gradients in one pass:
//   colour L1           sum |c - gt| / R                          model/training.py:506-509
//   eikonal             mean over samples of (|n|_2 - 1)^2         train.py:526
//   edge-aware smoothness of the depth within p x p patches        model/losses.py:20-38, train.py:519-525
//   plain smoothness                                                model/losses.py:7-18
// The torch expression of these terms launches ~150 small kernels per step
// (forward + autograd); here it is three launches.  Partial sums are reduced in
// double in a fixed order (deterministic); gradients follow autograd's rules
// (abs' = sign with sign(0) = 0, the norm's gradient is 0 at a zero vector).
#include "cn_common.h"

#include <algorithm>

namespace cn {

constexpr int kLossThreads = 256;
constexpr int kEikonalBlocks = 1024;

__device__ __forceinline__ float sgnf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

__device__ __forceinline__ double block_sum(double v, double* red) {
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int s = kLossThreads / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    return red[0];
}

// One thread per P x P patch of rays (the reference's d.view(-1, P, P, 1)):
// colour L1 of its P*P rays and the four neighbour-pair terms of both smoothness
// losses (losses.py:11-16, 30-37): horizontal (i, j)-(i, j+1), vertical
// (i, j)-(i+1, j), diagonal (i, j)-(i+1, j+1), anti-diagonal (i+1, j)-(i, j+1).
// Each pair type is a mean over npatch * (pairs per patch) elements and the four
// means are averaged (/ 4).  P = 1: colour L1 only.
template <int P>
__global__ void __launch_bounds__(kLossThreads) patch_loss_kernel(int npatch, const float* __restrict__ color,
                                                                  const float* __restrict__ gt,
                                                                  const float* __restrict__ depth,
                                                                  const float* __restrict__ wts, float gamma, int R,
                                                                  float* dcolor, float* ddepth, double* part) {
    __shared__ double red[kLossThreads];
    constexpr int Q = P * P;
    const float w_rgb = wts[0], w_edge = wts[2], w_smooth = wts[3];
    const int p = blockIdx.x * kLossThreads + threadIdx.x;
    double acc = 0.0;
    if (p < npatch) {
        const int r0 = p * Q;
        float d[Q], g[Q][3], dd[Q];
        double l1 = 0.0;
        const float crgb = w_rgb / (float)R;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            d[q] = depth[r0 + q];
            dd[q] = 0.0f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                g[q][c] = gt[3 * (r0 + q) + c];
                const float x = color[3 * (r0 + q) + c] - g[q][c];
                l1 += (double)fabsf(x);
                dcolor[3 * (r0 + q) + c] = sgnf(x) * crgb;
            }
        }
        acc += (double)w_rgb * l1 / (double)R;
        if constexpr (P >= 2) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int cnt = t < 2 ? P * (P - 1) : (P - 1) * (P - 1);
                const double n = (double)npatch * cnt;
                const float ce = (float)(0.25 * w_edge / n), cs = (float)(0.25 * w_smooth / n);
                double se = 0.0, ss = 0.0;
#pragma unroll
                for (int i = 0; i < P; ++i)
#pragma unroll
                    for (int j = 0; j < P; ++j) {
                        int a, b;
                        if (t == 0) {
                            if (j == P - 1) continue;
                            a = i * P + j, b = i * P + j + 1;
                        } else if (t == 1) {
                            if (i == P - 1) continue;
                            a = i * P + j, b = (i + 1) * P + j;
                        } else if (t == 2) {
                            if (i == P - 1 || j == P - 1) continue;
                            a = i * P + j, b = (i + 1) * P + j + 1;
                        } else {
                            if (i == P - 1 || j == P - 1) continue;
                            a = (i + 1) * P + j, b = i * P + j + 1;
                        }
                        const float diff = d[a] - d[b];
                        // bilateral weight exp(-sum_c |img_a - img_b| / gamma) (losses.py:27-28)
                        const float sad =
                            (fabsf(g[a][0] - g[b][0]) + fabsf(g[a][1] - g[b][1])) + fabsf(g[a][2] - g[b][2]);
                        const float bw = expf(-sad / gamma);
                        se += (double)fabsf(bw * diff);
                        ss += (double)fabsf(diff);
                        const float s = sgnf(diff);
                        const float gd = ce * bw * s + cs * s;
                        dd[a] += gd;
                        dd[b] -= gd;
                    }
                acc += 0.25 * ((double)w_edge * se + (double)w_smooth * ss) / n;
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) ddepth[r0 + q] = dd[q];
    }
    const double tot = block_sum(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// Eikonal term over every sample: (|n| - 1)^2, gradient coef * 2 (|n| - 1) n / |n|, coef = w_eik / M.
__global__ void __launch_bounds__(kLossThreads) eikonal_kernel(int64_t M, const float* __restrict__ nrm, int64_t ldn,
                                                               const float* __restrict__ wts, float* dn, int64_t ld_dn,
                                                               double* part) {
    __shared__ double red[kLossThreads];
    const float coef = wts[1] / (float)M;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kLossThreads;
    for (int64_t m = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; m < M; m += stride) {
        const float x = nrm[m * ldn], y = nrm[m * ldn + 1], z = nrm[m * ldn + 2];
        const float r = sqrtf(x * x + y * y + z * z);
        const float e = r - 1.0f;
        acc += (double)(e * e);
        const float g = r > 0.0f ? coef * 2.0f * e / r : 0.0f;
        dn[m * ld_dn] = g * x;
        dn[m * ld_dn + 1] = g * y;
        dn[m * ld_dn + 2] = g * z;
    }
    const double tot = block_sum(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// loss = sum(part_a) + (w_eik / M) sum(part_b), each summed in a fixed order.  The
// device-side NaN guard of model/training.py:532-533 (assert not torch.isnan(loss)):
// a non-finite loss sets the sticky flag *nonfinite, which the host reads when it
// syncs anyway -- no per-step host sync, so the step stays graph-capturable.
__global__ void __launch_bounds__(kLossThreads) loss_finalize_kernel(const double* part_a, int na,
                                                                     const double* part_b, int nb, int64_t M,
                                                                     const float* __restrict__ wts, float* loss,
                                                                     int* nonfinite) {
    __shared__ double red[kLossThreads];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < na; i += kLossThreads) a += part_a[i];
    for (int i = threadIdx.x; i < nb; i += kLossThreads) b += part_b[i];
    const double sa = block_sum(a, red);
    __syncthreads();
    const double sb = block_sum(b, red);
    if (threadIdx.x == 0) {
        const double coef_b = M > 0 ? (double)wts[1] / (double)M : 0.0;
        const float l = (float)(sa + coef_b * sb);
        *loss = l;
        if (nonfinite && !isfinite(l)) *nonfinite = 1;
    }
}

// patch threads (patches, or rays for P = 1) and their workgroups
static int loss_units(int R, int patch) { return patch >= 2 ? R / (patch * patch) : R; }
static int loss_blocks(int R, int patch) { return std::max(1, cdiv(loss_units(R, patch), kLossThreads)); }

}  // namespace cn

using namespace cn;

extern "C" size_t cn_train_loss_workspace_bytes(int32_t R, int32_t patch) {
    return sizeof(double) * ((size_t)loss_blocks(std::max(R, 1), std::max(patch, 1)) + kEikonalBlocks);
}

extern "C" int cn_train_loss(int32_t R, int32_t patch, int64_t M, const float* color, const float* gt,
                             const float* depth, const float* normals, int64_t ld_n, const float* weights,
                             float gamma, float* loss, float* dcolor, float* ddepth, float* dnormals, int64_t ld_dn,
                             int32_t* nonfinite, void* workspace, int64_t workspace_bytes, cn_stream_t stream) {
    CN_REQUIRE(color && gt && depth && weights && loss && dcolor && ddepth && workspace, CN_ERR_ARG,
               "cn_train_loss: null pointer");
    CN_REQUIRE(R > 0 && M >= 0 && (M == 0 || (normals && dnormals && ld_n >= 3 && ld_dn >= 3)), CN_ERR_SHAPE,
               "cn_train_loss: bad R=%d / M=%lld / normals", R, (long long)M);
    CN_REQUIRE(patch >= 1 && patch <= 4 && R % (patch * patch) == 0, CN_ERR_UNSUPPORTED,
               "cn_train_loss: patch %d (1..4, R a multiple of patch^2)", patch);
    CN_REQUIRE(gamma > 0.0f, CN_ERR_ARG, "cn_train_loss: gamma must be positive");
    CN_REQUIRE((size_t)workspace_bytes >= cn_train_loss_workspace_bytes(R, patch), CN_ERR_SHAPE,
               "cn_train_loss: workspace");
    hipStream_t s = (hipStream_t)stream;
    double* part_a = static_cast<double*>(workspace);
    const int na = loss_blocks(R, patch), nu = loss_units(R, patch);
    double* part_b = part_a + na;
    switch (patch) {
        case 1: patch_loss_kernel<1><<<na, kLossThreads, 0, s>>>(nu, color, gt, depth, weights,
                                                                  gamma, R, dcolor, ddepth, part_a); break;
        case 2: patch_loss_kernel<2><<<na, kLossThreads, 0, s>>>(nu, color, gt, depth, weights,
                                                                  gamma, R, dcolor, ddepth, part_a); break;
        case 3: patch_loss_kernel<3><<<na, kLossThreads, 0, s>>>(nu, color, gt, depth, weights,
                                                                  gamma, R, dcolor, ddepth, part_a); break;
        default: patch_loss_kernel<4><<<na, kLossThreads, 0, s>>>(nu, color, gt, depth, weights,
                                                                   gamma, R, dcolor, ddepth, part_a); break;
    }
    int rc = check_launch("cn_train_loss (patch terms)");
    if (rc) return rc;
    int nb = 0;
    if (M > 0) {
        nb = (int)std::min<int64_t>(kEikonalBlocks, (M + kLossThreads - 1) / kLossThreads);
        eikonal_kernel<<<nb, kLossThreads, 0, s>>>(M, normals, ld_n, weights, dnormals, ld_dn, part_b);
        rc = check_launch("cn_train_loss (eikonal)");
        if (rc) return rc;
    }
    loss_finalize_kernel<<<1, kLossThreads, 0, s>>>(part_a, na, part_b, nb, M, weights, loss, nonfinite);
    return check_launch("cn_train_loss (finalize)");
}
