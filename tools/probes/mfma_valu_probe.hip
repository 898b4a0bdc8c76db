// Probe: can a wave's f32 VALU stream run beside a partner wave's
// v_mfma_f32_32x32x2_f32 stream on the same SIMD?  512-thread blocks, one per
// CU: waves 0-3 (one per SIMD) run NM MFMAs, waves 4-7 run NV independent FMAs.
// Also: MFMA + NV_IN VALU per MFMA interleaved inside one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NVIN>
__global__ void __launch_bounds__(512) probe(float* out, int nm, int nv) {
    constexpr int nv_in = NVIN;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    float a = lane * 1e-3f, b = 1.0f - lane * 1e-3f;
    if (wave < 4) {
        if (nm == 0) return;
        floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        float v[8];
        for (int q = 0; q < 8; ++q) v[q] = lane + q;
        for (int i = 0; i < nm; i += 4) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < nv_in; ++r) v[r & 7] = __builtin_fmaf(v[r & 7], 1.0001f, 0.5f);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c1, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < nv_in; ++r) v[r & 7] = __builtin_fmaf(v[r & 7], 1.0001f, 0.5f);
            c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c2, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < nv_in; ++r) v[r & 7] = __builtin_fmaf(v[r & 7], 1.0001f, 0.5f);
            c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c3, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < nv_in; ++r) v[r & 7] = __builtin_fmaf(v[r & 7], 1.0001f, 0.5f);
        }
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
        for (int q = 0; q < 8; ++q) s += v[q];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    } else {
        if (nv == 0) return;
        float v[8];
        for (int q = 0; q < 8; ++q) v[q] = lane + q;
        for (int i = 0; i < nv; i += 8) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = __builtin_fmaf(v[q], 1.0001f, 0.5f);
        }
        float s = 0.f;
        for (int q = 0; q < 8; ++q) s += v[q];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    }
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * 512 * cus);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int NM = 4096;
    struct { int nm, nv, nv_in; const char* what; } cfg[] = {
        {NM, 0, 0, "MFMA only (waves 0-3)"},
        {0, NM * 16, 0, "VALU only (waves 4-7), 16 FMA per MFMA-equivalent"},
        {NM, NM * 16, 0, "MFMA waves + VALU partner waves (16 FMA/MFMA)"},
        {0, NM * 8, 0, "VALU only, 8 FMA per MFMA-equivalent"},
        {NM, NM * 8, 0, "MFMA + VALU partner (8 FMA/MFMA)"},
        {NM, 0, 4, "MFMA with 4 FMA interleaved in-wave"},
        {NM, 0, 8, "MFMA with 8 FMA interleaved in-wave"},
        {NM, 0, 16, "MFMA with 16 FMA interleaved in-wave"},
    };
    for (auto& c : cfg) {
        auto run = [&] {
            if (c.nv_in == 0) probe<0><<<cus, 512>>>(out, c.nm, c.nv);
            else if (c.nv_in == 4) probe<4><<<cus, 512>>>(out, c.nm, c.nv);
            else if (c.nv_in == 8) probe<8><<<cus, 512>>>(out, c.nm, c.nv);
            else probe<16><<<cus, 512>>>(out, c.nm, c.nv);
        };
        run();
        hipEventRecord(e0);
        run();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-55s %8.1f us  (%.1f ns per MFMA-slot)\n", c.what, ms * 1e3, ms * 1e6 / NM);
    }
    (void)hipFree(out);
    return 0;
}
