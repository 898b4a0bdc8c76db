// cn_pack.hip — weight images for cn_linear, one launch per network.
//
// Every call of the SDF / colour networks packs its effective (weight-normed)
// weights into zero-padded GEMM images: forward [N][K], transposed [K][N] for
// the adjoint passes, the colour network's first layer with its columns
// permuted to [feature | gradient | point | view encoding], and, in bf16x6
// mode, the three bf16 terms of every value.  As torch ops that is ~9 launches
// per image and ~27 images per step; here it is one launch whose jobs (one per
// image region) travel as the kernel argument.
#include "cn_common.h"

#include <algorithm>

namespace cn {

constexpr int kPackJobsPerLaunch = 24;  // 24 x 56 B of kernel arguments

struct PackBatch {
    cn_pack_job job[kPackJobsPerLaunch];
};

// The same three RNE roundings as ops.split_bf16x3 (torch .to(bfloat16)), so
// both builders give bit-identical images.
__device__ __forceinline__ unsigned short bf16_rne(float x) {
    return __builtin_bit_cast(unsigned short, static_cast<__bf16>(x));
}
__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
    return __builtin_bit_cast(float, static_cast<unsigned>(h) << 16);
}

// grid: (blocks per job, jobs); each block strides over its job's region with
// the column index fastest (coalesced stores; transposed sources are small and
// L2-resident).
__global__ void __launch_bounds__(256) pack_kernel(PackBatch b) {
    const cn_pack_job& j = b.job[blockIdx.y];
    const int w = j.c1 - j.c0;
    const int64_t n = (int64_t)(j.r1 - j.r0) * w;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int rr = (int)(e / w), cc = (int)(e % w);
        float v = 0.0f;
        if (rr < j.rows && cc < j.cols) v = j.transpose ? j.src[(int64_t)cc * j.src_ld + rr] : j.src[(int64_t)rr * j.src_ld + cc];
        const int64_t r = j.r0 + rr, c = j.c0 + cc;
        if (j.format == CN_MFMA_F32) {
            static_cast<float*>(j.dst)[r * j.dst_ld + c] = v;
        } else if (j.format == CN_MFMA_BF16) {
            static_cast<unsigned short*>(j.dst)[r * j.dst_ld + c] = bf16_rne(v);
        } else {
            // chunk-major term image: (c / 16, r, t, c % 16), dst_ld = image rows
            unsigned short* d = static_cast<unsigned short*>(j.dst) + ((c >> 4) * j.dst_ld + r) * 48 + (c & 15);
            const unsigned short t0 = bf16_rne(v);
            const float q = v - bf16_to_f32(t0);
            const unsigned short t1 = bf16_rne(q);
            const unsigned short t2 = bf16_rne(q - bf16_to_f32(t1));
            d[0] = t0;
            d[16] = t1;
            d[32] = t2;
        }
    }
}

constexpr int kWnJobsPerLaunch = 16;
struct WnBatch {
    cn_wn_job job[kWnJobsPerLaunch];
};

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// grid (row blocks, jobs), 256 threads = 4 waves = 4 rows per block.
__global__ void __launch_bounds__(256) weight_norm_kernel(WnBatch b, int backward) {
    const cn_wn_job& j = b.job[blockIdx.y];
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= j.rows) return;
    const float* v = j.v + (int64_t)row * j.cols;
    float ss = 0.0f;
    for (int c = lane; c < j.cols; c += 64) ss += v[c] * v[c];
    const float nrm = sqrtf(wave_sum(ss));
    const float g = j.g[row];
    if (!backward) {
        const float s = g / nrm;
        float* w = j.w + (int64_t)row * j.cols;
        for (int c = lane; c < j.cols; c += 64) w[c] = v[c] * s;
        return;
    }
    const float* dw = j.dw + (int64_t)row * j.cols;
    float dot = 0.0f;
    for (int c = lane; c < j.cols; c += 64) dot += dw[c] * v[c];
    dot = wave_sum(dot);
    const float dg = dot / nrm;
    if (lane == 0) j.dg[row] = dg;
    const float s = g / nrm, t = dg / nrm;
    float* dv = j.dv + (int64_t)row * j.cols;
    for (int c = lane; c < j.cols; c += 64) dv[c] = s * (dw[c] - v[c] * t);
}

}  // namespace cn

using namespace cn;

extern "C" int cn_weight_norm(const cn_wn_job* jobs, int32_t njobs, int32_t backward, cn_stream_t stream) {
    CN_REQUIRE(njobs >= 0 && (jobs || njobs == 0), CN_ERR_ARG, "cn_weight_norm: bad job list");
    for (int i = 0; i < njobs; ++i) {
        const cn_wn_job& j = jobs[i];
        CN_REQUIRE(j.v && j.g && (backward ? (j.dw && j.dv && j.dg) : (j.w != nullptr)), CN_ERR_ARG,
                   "cn_weight_norm: job %d null pointer", i);
        CN_REQUIRE(j.rows >= 0 && j.cols >= 0, CN_ERR_SHAPE, "cn_weight_norm: job %d shape", i);
    }
    for (int i0 = 0; i0 < njobs; i0 += kWnJobsPerLaunch) {
        const int n = njobs - i0 < kWnJobsPerLaunch ? njobs - i0 : kWnJobsPerLaunch;
        WnBatch b{};
        int most = 0;
        for (int i = 0; i < n; ++i) {
            b.job[i] = jobs[i0 + i];
            most = std::max(most, b.job[i].rows);
        }
        if (most == 0) continue;
        weight_norm_kernel<<<dim3((most + 3) / 4, n), 256, 0, (hipStream_t)stream>>>(b, backward ? 1 : 0);
        const int rc = check_launch("cn_weight_norm");
        if (rc) return rc;
    }
    return CN_OK;
}

extern "C" int cn_pack_weights(const cn_pack_job* jobs, int32_t njobs, cn_stream_t stream) {
    CN_REQUIRE(njobs >= 0 && (jobs || njobs == 0), CN_ERR_ARG, "cn_pack_weights: bad job list");
    for (int i = 0; i < njobs; ++i) {
        const cn_pack_job& j = jobs[i];
        CN_REQUIRE(j.dst && (j.src || j.rows == 0 || j.cols == 0), CN_ERR_ARG, "cn_pack_weights: job %d null pointer", i);
        CN_REQUIRE(j.format == CN_MFMA_F32 || j.format == CN_MFMA_BF16 || j.format == CN_MFMA_F32_BF16X6, CN_ERR_ARG,
                   "cn_pack_weights: job %d bad format %d", i, j.format);
        CN_REQUIRE(0 <= j.r0 && j.r0 <= j.r1 && 0 <= j.c0 && j.c0 <= j.c1 && j.rows >= 0 && j.cols >= 0 &&
                       j.rows <= j.r1 - j.r0 && j.cols <= j.c1 - j.c0 &&
                       (j.format == CN_MFMA_F32_BF16X6 ? j.r1 <= j.dst_ld : j.c1 <= j.dst_ld) &&
                       (j.rows == 0 || j.cols == 0 || j.src_ld >= (j.transpose ? j.rows : j.cols)),
                   CN_ERR_SHAPE, "cn_pack_weights: job %d region [%d,%d)x[%d,%d) src %dx%d ld %lld dst ld %lld", i, j.r0,
                   j.r1, j.c0, j.c1, j.rows, j.cols, (long long)j.src_ld, (long long)j.dst_ld);
    }
    for (int i0 = 0; i0 < njobs; i0 += kPackJobsPerLaunch) {
        const int n = njobs - i0 < kPackJobsPerLaunch ? njobs - i0 : kPackJobsPerLaunch;
        PackBatch b{};
        int64_t most = 0;
        for (int i = 0; i < n; ++i) {
            b.job[i] = jobs[i0 + i];
            const int64_t e = (int64_t)(b.job[i].r1 - b.job[i].r0) * (b.job[i].c1 - b.job[i].c0);
            most = e > most ? e : most;
        }
        if (most == 0) continue;
        const int blocks = (int)std::min<int64_t>((most + 255) / 256, 128);
        pack_kernel<<<dim3(blocks, n), 256, 0, (hipStream_t)stream>>>(b);
        const int rc = check_launch("cn_pack_weights");
        if (rc) return rc;
    }
    return CN_OK;
}
