// cn_common.h — shared definitions for the cope-nerf MI355X (gfx950) kernels.
//
// Error model (include/copenerf.h): every extern "C" entry point validates its
// arguments on the host, launches on the caller's stream and returns 0 or a
// negative cn_status.  The message of the last failure on the calling thread is
// kept in a thread_local buffer (cn_last_error).  No entry point allocates,
// synchronises or touches the default stream, so a caller may capture any
// sequence of them into a hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>

#include "../../include/copenerf.h"

namespace cn {

void set_error(const char* fmt, ...);

// Check a launch; converts a HIP launch error into CN_ERR_LAUNCH.
int check_launch(const char* what);

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Column group g (4 columns) of the SDF positional encoding of x' = scale * x (neus_embedder.py:17-36:
// include_input, log bands, periodic_fns [sin, cos], d = 4): g 0 = x', g 1 + 2k = sin(2^k x'), g 2 + 2k
// = cos(2^k x') for k < L, zero for g >= 1 + 2L.  The one definition of the encoding: cn_sdf_embed and
// the first layer's fused operand load (cn_linear with emb_x) give the same bits.
__device__ __forceinline__ floatx4 sdf_embed_group(floatx4 xv, int g, int L, float scale) {
    floatx4 xs, o = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < 4; ++c) xs[c] = xv[c] * scale;
    if (g == 0) {
        o = xs;
    } else if (g < 1 + 2 * L) {
        const int k = (g - 1) >> 1;
        const float f = (float)(1 << k);
        const bool is_sin = ((g - 1) & 1) == 0;
        for (int c = 0; c < 4; ++c) {
            const float t = xs[c] * f;
            o[c] = is_sin ? sinf(t) : cosf(t);
        }
    }
    return o;
}
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ float sigmoidf_ref(float x) {
    // torch CPU sigmoid: 1 / (1 + exp(-x))
    return 1.0f / (1.0f + expf(-x));
}

// torch.nn.Softplus(beta, threshold): x if x*beta > threshold else log1p(exp(x*beta))/beta
__device__ __forceinline__ float softplus_ref(float x, float beta, float thr) {
    const float bx = x * beta;
    return bx > thr ? x : log1pf(expf(bx)) / beta;
}

// torch softplus_backward factor: 1 if x*beta > threshold else e/(e+1), e = exp(x*beta).
// For x*beta > ~16.6 the fp32 value is exactly 1, so the threshold branch and the
// sigmoid agree bit for bit; we keep torch's form.
__device__ __forceinline__ float softplus_grad_ref(float x, float beta, float thr) {
    const float bx = x * beta;
    if (bx > thr) return 1.0f;
    const float e = expf(bx);
    return e / (e + 1.0f);
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace cn

#define CN_REQUIRE(cond, code, ...)           \
    do {                                      \
        if (!(cond)) {                        \
            ::cn::set_error(__VA_ARGS__);     \
            return (code);                    \
        }                                     \
    } while (0)
