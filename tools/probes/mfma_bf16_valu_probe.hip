// Probe: does VALU (FMA, v_exp) run beside v_mfma_f32_32x32x16_bf16 on one SIMD?
// 512-thread blocks, one per CU.  Partner mode: waves 0-3 MFMA, waves 4-7 VALU.
// In-wave mode: NVIN independent VALU ops between consecutive MFMAs of one wave.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int NVIN, bool TRANS>
__global__ void __launch_bounds__(512) probe(float* out, int nm, int nv) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(lane * 1e-3f + i); b[i] = (__bf16)(1.0f - lane * 1e-3f); }
    auto valu = [&](float x) { return TRANS ? __builtin_amdgcn_exp2f(x * 0.999f) : __builtin_fmaf(x, 1.0001f, 0.5f); };
    if (wave < 4) {
        if (nm == 0) return;
        floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        float v[8];
        for (int q = 0; q < 8; ++q) v[q] = lane * 1e-3f + q * 1e-2f;
        for (int i = 0; i < nm; i += 4) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < NVIN; ++r) v[r & 7] = valu(v[r & 7]);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < NVIN; ++r) v[r & 7] = valu(v[r & 7]);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < NVIN; ++r) v[r & 7] = valu(v[r & 7]);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
            _Pragma("unroll") for (int r = 0; r < NVIN; ++r) v[r & 7] = valu(v[r & 7]);
        }
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
        for (int q = 0; q < 8; ++q) s += v[q];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    } else {
        if (nv == 0) return;
        float v[8];
        for (int q = 0; q < 8; ++q) v[q] = lane * 1e-3f + q * 1e-2f;
        for (int i = 0; i < nv; i += 8) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = valu(v[q]);
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
    const int NM = 8192;
    struct { int nm, nv, nv_in; bool trans; const char* what; } cfg[] = {
        {NM, 0, 0, false, "bf16 MFMA only (waves 0-3)"},
        {0, NM * 8, 0, false, "FMA only (waves 4-7), 8 per MFMA slot"},
        {NM, NM * 8, 0, false, "MFMA + FMA partner waves (8/MFMA)"},
        {0, NM * 2, 0, true, "v_exp only, 2 per MFMA slot"},
        {NM, NM * 2, 0, true, "MFMA + v_exp partner waves (2/MFMA)"},
        {NM, 0, 4, false, "MFMA + 4 FMA in-wave"},
        {NM, 0, 8, false, "MFMA + 8 FMA in-wave"},
        {NM, 0, 2, true, "MFMA + 2 v_exp in-wave"},
        {NM, 0, 4, true, "MFMA + 4 v_exp in-wave"},
    };
    for (auto& c : cfg) {
        auto run = [&] {
            if (c.trans) {
                if (c.nv_in == 0) probe<0, true><<<cus, 512>>>(out, c.nm, c.nv);
                else if (c.nv_in == 2) probe<2, true><<<cus, 512>>>(out, c.nm, c.nv);
                else probe<4, true><<<cus, 512>>>(out, c.nm, c.nv);
            } else {
                if (c.nv_in == 0) probe<0, false><<<cus, 512>>>(out, c.nm, c.nv);
                else if (c.nv_in == 4) probe<4, false><<<cus, 512>>>(out, c.nm, c.nv);
                else probe<8, false><<<cus, 512>>>(out, c.nm, c.nv);
            }
        };
        run();
        hipEventRecord(e0);
        run();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-45s %8.1f us  (%.2f ns per MFMA slot)\n", c.what, ms * 1e3, ms * 1e6 / NM);
    }
    (void)hipFree(out);
    return 0;
}
