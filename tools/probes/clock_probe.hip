// Probe: shader clock under a long f32-MFMA stream.  Wave 0 of every block
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz constant clock)
// around NM back-to-back v_mfma_f32_32x32x2_f32 on 4 independent accumulators.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) probe(float* out, unsigned long long* stamps, int nm) {
    const int lane = threadIdx.x & 63;
    float a = lane * 1e-3f, b = 1.0f - lane * 1e-3f;
    floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < nm; i += 4) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        stamps[4 * blockIdx.x] = t0;
        stamps[4 * blockIdx.x + 1] = t1;
        stamps[4 * blockIdx.x + 2] = r0;
        stamps[4 * blockIdx.x + 3] = r1;
    }
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    unsigned long long* st;
    (void)hipMalloc(&out, sizeof(float) * 256 * cus * 2);
    (void)hipMalloc(&st, sizeof(unsigned long long) * 4 * cus * 2);
    unsigned long long* h = new unsigned long long[4 * cus * 2];
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int nm : {4096, 65536, 262144}) {
        for (int wpc : {1, 2}) {  // blocks (of 4 waves) per CU
            const int grid = cus * wpc;
            probe<<<grid, 256>>>(out, st, nm);
            (void)hipEventRecord(e0);
            probe<<<grid, 256>>>(out, st, nm);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            (void)hipMemcpy(h, st, sizeof(unsigned long long) * 4 * grid, hipMemcpyDeviceToHost);
            double clk = 0;
            for (int bI = 0; bI < grid; ++bI)
                clk += (double)(h[4 * bI + 1] - h[4 * bI]) / ((double)(h[4 * bI + 3] - h[4 * bI + 2]) / 100e6);
            clk /= grid;
            const double tf = 2.0 * 32 * 32 * 2 * (double)nm * 4 * grid / (ms * 1e-3) / 1e12;
            printf("nm=%7d blocks/CU=%d  %9.1f us  %7.1f TFLOP/s  clock %.3f GHz  (cycles/MFMA/SIMD %.1f)\n", nm, wpc,
                   ms * 1e3, tf, clk / 1e9, clk * ms * 1e-3 / ((double)nm * wpc));
        }
    }
    return 0;
}
