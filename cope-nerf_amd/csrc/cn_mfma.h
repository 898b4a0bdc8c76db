// cn_mfma.h — device helpers shared by the MFMA GEMM kernels (cn_gemm.hip, cn_wgrad.hip):
// buffer-resource views, bf16x3 term splitting, softplus on the hardware transcendentals,
// XCD-aware tile order.
#pragma once

#include "cn_common.h"

namespace cn {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16_t;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

// Buffer views: every global access of the GEMM goes through a buffer resource
// whose base is a tile row and whose record count ends at the last valid row,
// so (a) per-access addressing is a per-lane 32-bit voffset fixed for the whole
// kernel plus a wave-uniform soffset (column offset) and SALU-built descriptors,
// no 64-bit VALU address math, and (b) rows >= M read as zero and their stores
// are dropped by the range check, with no per-row compare.  The range check
// covers voffset only (not soffset), so the row part of every offset is either
// in voffset or in the descriptor base.  On gfx950 the f32 MFMA and VALU instructions of the
// waves of one SIMD issue strictly one after the other (tools/probes), so every
// VALU instruction removed here is matrix-pipe time won back.
// bytes: a tile's extent, < 2^31 by the host's leading-dimension limit; <= 0 = empty view
__device__ __forceinline__ rsrc_t make_view(const float* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes < 0 ? 0 : bytes, 0x00020000);
}
// A tile's rows of one tensor: base = its first row, bytes = extent up to the last valid row.
struct TileView {
    const float* base;
    int ld;
    int bytes;
};
__device__ __forceinline__ rsrc_t view_at(const TileView& t, int lrow) {
    return make_view(t.base + (int64_t)lrow * t.ld, t.bytes - lrow * t.ld * 4);
}
__device__ __forceinline__ floatx4 bload4(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ float bload1(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// the value goes through a by-value parameter: __builtin_bit_cast applied directly
// to a vector element (acc[i][j][r]) miscompiles in ROCm 7.2 clang (every store
// of an unrolled loop gets element 0)
__device__ __forceinline__ void bstore1(rsrc_t r, int voff, int soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, 0);
}
__device__ __forceinline__ void bstore4(rsrc_t r, int voff, int soff, floatx4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, soff, 0);
}

// The epilogues' streams (aux rows read once, outputs written once) with a cache policy of their own:
// CN_EPI_AUX (measurement switch; 2 = nt on gfx950).
#ifndef CN_EPI_AUX
#define CN_EPI_AUX 2  // nt: measured faster (profiles/r6_ab.txt r6v)
#endif
__device__ __forceinline__ floatx4 eload4(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, CN_EPI_AUX));
}
__device__ __forceinline__ float eload1(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, CN_EPI_AUX));
}
// (bf16 aux rows keep the default policy: a 32-column block is half a 128-byte line, and nt loads do not
// allocate it in L2 for the neighbouring block's load -- measured slower, profiles/r6_ab.txt r6v)
__device__ __forceinline__ unsigned eload_u16(rsrc_t r, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
}
__device__ __forceinline__ void estore1(rsrc_t r, int voff, int soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, CN_EPI_AUX);
}
__device__ __forceinline__ void estore4(rsrc_t r, int voff, int soff, floatx4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, soff, CN_EPI_AUX);
}

// bf16 operand images (ABI v10): a tile's rows of a bf16 tensor (ld in bf16 elements, a
// multiple of 8) as the float-typed TileView over the same bytes (rows ld / 2 floats apart), so
// view_at works unchanged; voffsets into it are byte offsets, as for fp32 views.
__device__ __forceinline__ TileView tile_view_b16(const void* base, int ld, int64_t row0, int col0, int rows) {
    const char* b = static_cast<const char*>(base) + (row0 * ld + col0) * 2;
    return TileView{reinterpret_cast<const float*>(b), ld / 2, base ? (rows * ld - col0) * 2 : 0};
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
// one bf16 read as the fp32 value it represents
__device__ __forceinline__ float bload_b16(rsrc_t r, int voff, int soff) {
    const unsigned short h = __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
    return __builtin_bit_cast(float, (unsigned)h << 16);
}
// one bf16 as its raw bits (zero-extended)
__device__ __forceinline__ unsigned bload_u16(rsrc_t r, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
}
// four bf16 (8 bytes) as fp32 values
__device__ __forceinline__ floatx4 bload_b16x4(rsrc_t r, int voff, int soff) {
    const u32x2_t w = __builtin_bit_cast(u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    return floatx4{__builtin_bit_cast(float, w[0] << 16), __builtin_bit_cast(float, w[0] & 0xffff0000u),
                   __builtin_bit_cast(float, w[1] << 16), __builtin_bit_cast(float, w[1] & 0xffff0000u)};
}
// RNE bf16 of two / four fp32 values (v_cvt_pk_bf16_f32: the rounding the GEMM staging applies)
__device__ __forceinline__ unsigned pack_b16x2(float a, float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, bf16x2_t));
}
__device__ __forceinline__ void bstore_b16x2(rsrc_t r, int voff, int soff, float a, float b) {
    __builtin_amdgcn_raw_buffer_store_b32(pack_b16x2(a, b), r, voff, soff, 0);
}
__device__ __forceinline__ void bstore_b16x4(rsrc_t r, int voff, int soff, floatx4 v) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    const b4 h = __builtin_convertvector(v, b4);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, h), r, voff, soff, 0);
}

// torch.nn.Softplus(beta, threshold) on the hardware transcendentals: e = 2^(z beta
// log2 e), a = log2(1 + e) ln2 / beta; the linear branch (beta z > threshold) exactly
// as torch.  Absolute error of a is ~1e-9 (log2 of the rounded 1 + e; v_exp/v_log
// are 1 ulp), far below the fp32 GEMM rounding of the layer that produced z.
__device__ __forceinline__ float softplus_hw(float z, float c_exp, float c_thr, float c_log) {
    const float y = z * c_exp;  // beta z log2(e)
    const float e = __builtin_amdgcn_exp2f(y);
    const bool lin = y > c_thr;  // beta z > threshold (boundary moved by <= 1 ulp; the branches agree to 1e-10 there)
    return lin ? z : __builtin_amdgcn_logf(1.0f + e) * c_log;
}

// softplus'(z) = sigmoid(beta z) recovered from the softplus output a = softplus(z):
// exp(beta a) = 1 + exp(beta z), so sigma = 1 - exp(-beta a) (= 1 exactly in fp32 on
// torch's linear branch, beta z > 20).  aux_c = -beta * log2(e) (times the divisor the
// stored activation carries).  Absolute error <= ~1e-7: the backward never stores
// sigma, every consumer reads the activation it already has.
__device__ __forceinline__ float sigma_from_act(float a, float aux_c) {
    return 1.0f - __builtin_amdgcn_exp2f(a * aux_c);
}

// Three-term bf16 split of 4 fp32 values (CN_MFMA_F32_BF16X6): v = t0 + t1 + t2
// with every term the RNE bf16 of the remainder.  Written on packed pairs: the
// bf16 -> fp32 widening of a v_cvt_pk_bf16_f32 result is a shift (low half) and
// a mask (high half), the remainders scalar v_sub_f32 (sub_f32): 20 VALU per 4 values
// (the per-element convertvector round trip compiles to 30).
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ floatx2 widen_bf16x2(unsigned p) {
    return floatx2{__builtin_bit_cast(float, p << 16), __builtin_bit_cast(float, p & 0xffff0000u)};
}
// x - y as one v_sub_f32 (exact here: the remainders are representable).  Written as asm so the
// compiler cannot pair two of them into a v_pk_add_f32, which beside the MFMAs costs several times the
// issue cycles of two scalar ones (MI355X_MICROARCH.md, issue-cost rows).
__device__ __forceinline__ float sub_f32(float x, float y) {
#if CN_SPLIT_PK
    return x - y;
#else
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
#endif
}
__device__ __forceinline__ float add_f32(float x, float y) {
#if CN_SPLIT_PK
    return x + y;
#else
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
#endif
}
__device__ __forceinline__ void split3(floatx4 v, bf16x4& t0, bf16x4& t1, bf16x4& t2) {
    unsigned p0[2], p1[2], p2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const floatx2 x = {v[2 * h], v[2 * h + 1]};
        p0[h] = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
        const floatx2 w0 = widen_bf16x2(p0[h]);
        const floatx2 r = {sub_f32(x[0], w0[0]), sub_f32(x[1], w0[1])};
        p1[h] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
        const floatx2 w1 = widen_bf16x2(p1[h]);
        const floatx2 q = {sub_f32(r[0], w1[0]), sub_f32(r[1], w1[1])};
        p2[h] = __builtin_bit_cast(unsigned, __builtin_convertvector(q, bf16x2));
    }
    t0 = __builtin_bit_cast(bf16x4, (u32x2){p0[0], p0[1]});
    t1 = __builtin_bit_cast(bf16x4, (u32x2){p1[0], p1[1]});
    t2 = __builtin_bit_cast(bf16x4, (u32x2){p2[0], p2[1]});
}

// s_waitcnt that waits for this wave's vector-memory count to drop to N (expcnt, lgkmcnt untouched).
// The LDS-DMA rings wait with it: the compiler would otherwise drain every DMA in flight.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// 16-byte LDS read as inline asm (the caller waits lgkmcnt): beside an LDS-DMA ring a compiled
// LDS read would make the compiler drain every DMA in flight first (vmcnt(0)), since it cannot
// tell the ring's buffers apart.
template <int OFF>
__device__ __forceinline__ u32x4 lds_read_b128(uint32_t addr) {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
    return r;
}

// Virtual tile vt -> (tm, tn).  XCD-aware: blocks b and b+8 are dispatched to
// the same XCD, so the T N-tiles of one M-tile are placed 8 apart and share that
// XCD's L2 copy of the A rows.  Tiles are padded to a multiple of 8 M-tiles.
__device__ __forceinline__ void tile_coords(int vt, int T, int& tm, int& tn) {
    const int grp = vt / (8 * T);
    const int w = vt % (8 * T);
    tm = grp * 8 + (w & 7);
    tn = w >> 3;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline bool al8(const void* p) { return ((uintptr_t)p & 7) == 0; }

// Fixed-order sum of nslab fp32 slabs (cn_wgrad.hip): out[r*ldo + c] (+)= (sum_s part[s*stride + r*ldp + c]) / div.
struct SlabJob {
    const float* part;
    float* out;
    int64_t stride, ldp, ldo;
    int nslab, rows, cols, accumulate, blocks;
    float div;
};
SlabJob slab_job(const float* part, int nslab, int64_t stride, int rows, int cols, int64_t ldp, float* out,
                 int64_t ldo, float div, int accumulate);
// up to kSlabMax reductions in one launch: workgroups [blk0[i], blk0[i] + j[i].blocks) take job i
constexpr int kSlabMax = 32;
struct SlabBatch {
    SlabJob j[kSlabMax];
    int n;
};
// two reductions in one launch (j1 may be SlabJob{}: empty)
int launch_slab_jobs(const SlabJob& j0, const SlabJob& j1, hipStream_t s);
int launch_slab_batch(const SlabJob* jobs, int n, hipStream_t s);
int launch_slab_reduce(const float* part, int nslab, int64_t stride, int rows, int cols, int64_t ldp, float* out,
                       int64_t ldo, float div, int accumulate, hipStream_t s);

}  // namespace cn
