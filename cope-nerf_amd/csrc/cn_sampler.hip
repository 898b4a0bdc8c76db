// cn_sampler.hip — the sampler's SDF query as one kernel (gfx950, bf16 MLP mode).
//
// NeuSRenderer.up_sample (model/neus_renderer.py:492-525) queries SDFNetwork.sdf at the coarse
// samples and at every round's new samples with no gradient: embedding (neus_embedder.py:17-36),
// eight softplus layers with the skip concat (neus_fields.py:268-283) and the sdf row of the last
// Linear.  Layer by layer that is nine launches whose activations go through HBM (~8 KB per sample
// in bf16 images).  Here one persistent workgroup per CU takes 256 samples at a time through all
// nine layers and writes only the sdf:
//
//  * activations stay in registers.  Each wave owns 64 samples and ALL 256 features, computing
//    outᵀ = W · actᵀ: the weights are the MFMA A operand, the activations the B operand.  A 32x32
//    accumulator block then holds one sample per lane and 16 features in registers, and after the
//    layer's epilogue (bias, softplus, RNE bf16) two v_permlane32_swap per 8 values put them in the
//    next layer's B-operand order (lane half h: features 8h .. 8h + 7 of each 16-deep k-step).  No
//    LDS and no HBM between layers.
//  * weights stream through an LDS-DMA ring: 32-deep chunks of a layer's [256][K] bf16 image (16 KB,
//    64-byte rows XOR-swizzled by (row >> 2) & 3 in the source address), 8 slots, 7 chunks in
//    flight across layer and sample-block boundaries; every wave reads every chunk (4 waves share
//    each weight byte fetched from L2).
//  * per sample: the embedding's bf16 image in (lin0's input, 128 B, and the skip concat's tail, E
//    values; cn_sdf_embed writes both, as for the layer-by-layer path) and the sdf (4 B) out.  (The
//    embedding's sinf / cosf inlined here took the registers the chain needs: spills.)
//
// Bitwise equal to the layer-by-layer bf16 path (sdf_forward on bf16 images: cn_sdf_embed, the
// 128x128 K = 64 tile, the 256x256 SOFTPLUS tiles, the SOFTPLUS_HEAD row-dot): the same RNE
// roundings, the same k order of the same MFMA per output (operands swapped), the same softplus
// instructions, and the head's row sum in the DMA tile's order (per column block, then the 32-lane
// butterfly, then the two column halves).
#include "cn_mfma.h"

#include <utility>

namespace cn {

// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled by construction (register arrays indexed by
// I stay in registers; a loop the compiler declines to unroll would send them to scratch)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int kMlpLayers = 8;       // lin0 .. lin7 (lin8's sdf row is the head)
constexpr int kMlpNS = 8;           // weight ring slots
constexpr int kMlpChunk = 16384;    // bytes per slot: 256 rows x 32 k bf16
constexpr int kMlpChunksPerBlock = 2 + 7 * 8;  // K = 64 for lin0, 256 for lin1..lin7

struct SdfMlpArgs {
    const bf16_t* u0;                 // [M][ld_u0] bf16: the embedding, 64 columns (lin0's input)
    const bf16_t* tail;               // [M][ld_t] bf16: the embedding / u4div (the skip layer's tail)
    int ld_u0, ld_t, M, nblocks;
    const bf16_t* W[kMlpLayers];      // weight images [256][K] (K = 64 for lin0, 256 else), rows >= N zero
    int ldw[kMlpLayers];
    const float* bias[kMlpLayers];
    int nout[kMlpLayers];             // 256, or (the skip layer) 256 - E
    float inv_odiv[kMlpLayers];       // 1, or 1/sqrt(2) for the layer feeding the skip concat
    const float* head_w;              // [256] sdf row of lin8 / scale
    const float* head_b;              // [1]
    float* sdf;
    const int* idx;                   // scatter: sdf[idx[m]] (or NULL: sdf[m])
    int skip_layer;                   // the layer whose columns >= nout carry the tail
    float beta, threshold;
    bf16_t* dbg;                      // (DBG) every layer's input, [8][M][256] natural feature order
};

template <bool DBG>
__global__ void __launch_bounds__(256, 1) sdf_mlp_kernel(SdfMlpArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[kMlpNS * kMlpChunk + kMlpLayers * 256 * 4 + 256 * 4];
    float* sBias = reinterpret_cast<float*>(smem + kMlpNS * kMlpChunk);
    float* sHead = sBias + kMlpLayers * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l31 = lane & 31;

    // bias tables and head weights (zero past each layer's width)
    for (int i = tid; i < kMlpLayers * 256; i += 256) {
        const int l = i >> 8, n = i & 255;
        sBias[i] = n < p.nout[l] ? p.bias[l][n] : 0.0f;
    }
    sHead[tid] = p.head_w[tid];
    __syncthreads();

    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
    const uint32_t ldsBias = lds0 + kMlpNS * kMlpChunk;
    const uint32_t ldsHead = ldsBias + kMlpLayers * 256 * 4;

    // ---- weight chunk stream: chunk g of the workgroup's stream is chunk g % 58 of a sample block
    auto chunk_of = [](int cb, int& l, int& k0) __attribute__((always_inline)) {
        if (cb < 2) {
            l = 0;
            k0 = 32 * cb;
        } else {
            l = 1 + ((cb - 2) >> 3);
            k0 = 32 * ((cb - 2) & 7);
        }
    };
    // wave w fills rows 64w .. 64w + 63 of the slot: four 1 KB pieces of 16 rows; lane l -> row
    // + (l >> 2), physical 16-byte chunk l & 3 (logical chunk (l & 3) ^ ((row >> 2) & 3))
    auto issue = [&](int g) __attribute__((always_inline)) {
        int l, k0;
        chunk_of(g % kMlpChunksPerBlock, l, k0);
        const int ldw = p.ldw[l];
        const rsrc_t v = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.W[l]), 0, 256 * ldw * 2, 0x00020000);
        char* dst = smem + (g % kMlpNS) * kMlpChunk + wave * 64 * 64;
        // (row >> 2) & 3 = (lane >> 4) & 3: the lane's part of the address is one VGPR, the rest soffset
        const int vo = ((lane >> 2) * ldw + 8 * ((lane & 3) ^ ((lane >> 4) & 3))) * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(v, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16, vo,
                                                     ((wave * 64 + 16 * j) * ldw + k0) * 2, 0, 0);
    };
    // A-operand (weight) reads: lane l -> row (l & 31) of each 32-row block, logical chunk 2s + h
    uint32_t aoff[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) aoff[s] = l31 * 64 + (((2 * s + h) ^ ((l31 >> 2) & 3)) << 4);

    const float c_exp = p.beta * 1.44269504088896341f;
    const float c_thr = p.threshold * 1.44269504088896341f;
    const float c_log = 0.693147180559945309f / p.beta;

    // ---- samples: wave w owns samples 64w + 32jb + (lane & 31) of the block
    const rsrc_t vu = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.u0), 0, p.M * p.ld_u0 * 2, 0x00020000);
    const rsrc_t vt = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.tail), 0, p.M * p.ld_t * 2, 0x00020000);
    const rsrc_t vi = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.idx), 0, p.idx ? p.M * 4 : 0, 0x00020000);
    int is[2];

    int blk = blockIdx.x;
    if (blk >= p.nblocks) return;
    int g = 0;  // the stream position of the current chunk
#pragma unroll
    for (int d = 0; d < kMlpNS - 1; ++d) issue(d);

    bf16x8 bq[2][16];  // the current layer's input: [sample block][k-step], B-operand order
    floatx16 acc[8][2];
    // (DBG) layer l's input as the B operand holds it: lane half h of k-step ks = features 16 ks + 8 h ..
    auto dump = [&](int l, int nks) __attribute__((always_inline)) {
        if constexpr (DBG) {
            for (int jb = 0; jb < 2; ++jb) {
                const int m = blk * 256 + wave * 64 + 32 * jb + l31;
                if (m < p.M)
#pragma unroll
                    for (int ks = 0; ks < 16; ++ks)
                        if (ks < nks)
                            *reinterpret_cast<bf16x8*>(p.dbg + ((int64_t)l * p.M + m) * 256 + 16 * ks + 8 * h) = bq[jb][ks];
            }
        }
    };

    // one 32-deep weight chunk (stream position g, k-steps 2q, 2q + 1 of the layer)
    auto chunk = [&](auto q_c) __attribute__((always_inline)) {
        constexpr int q = decltype(q_c)::value;
        // chunk g landed (this wave's pieces: DNS - 2 later chunks, 4 pieces each, were issued after
        // them), then every wave's; the slot of chunk g - 1 is free
        wait_vmcnt<4 * (kMlpNS - 2)>();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(g + kMlpNS - 1);
        const uint32_t sb = lds0 + (g % kMlpNS) * kMlpChunk;
        // one k-step's 8 A fragments at a time (the second step's reads go out behind the first step's
        // 16 MFMAs: 32 VGPRs instead of 64)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const uint32_t a = sb + aoff[s];
            bf16x8 af[8];
            af[0] = __builtin_bit_cast(bf16x8, lds_read_b128<0 * 2048>(a));
            af[1] = __builtin_bit_cast(bf16x8, lds_read_b128<1 * 2048>(a));
            af[2] = __builtin_bit_cast(bf16x8, lds_read_b128<2 * 2048>(a));
            af[3] = __builtin_bit_cast(bf16x8, lds_read_b128<3 * 2048>(a));
            af[4] = __builtin_bit_cast(bf16x8, lds_read_b128<4 * 2048>(a));
            af[5] = __builtin_bit_cast(bf16x8, lds_read_b128<5 * 2048>(a));
            af[6] = __builtin_bit_cast(bf16x8, lds_read_b128<6 * 2048>(a));
            af[7] = __builtin_bit_cast(bf16x8, lds_read_b128<7 * 2048>(a));
            asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3]));
#pragma unroll
            for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                for (int jb = 0; jb < 2; ++jb)
                    acc[ib][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ib], bq[jb][2 * q + s], acc[ib][jb], 0, 0, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[4]), "+v"(af[5]), "+v"(af[6]), "+v"(af[7]));
#pragma unroll
            for (int ib = 4; ib < 8; ++ib)
#pragma unroll
                for (int jb = 0; jb < 2; ++jb)
                    acc[ib][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ib], bq[jb][2 * q + s], acc[ib][jb], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        ++g;
    };
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int ib = 0; ib < 8; ++ib)
#pragma unroll
            for (int jb = 0; jb < 2; ++jb)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[ib][jb][r] = 0.0f;
    };
    // 4 x 4 consecutive floats of an LDS table, features 32 ib + 8 rq + 4 h .. + 3 (rq = 0..3): one base
    // register per half, the rest immediates
    auto read4 = [&](uint32_t base, auto ib_c, floatx4* v) __attribute__((always_inline)) {
        constexpr int ib = decltype(ib_c)::value;
        const uint32_t a = base + 16 * h;
        v[0] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 0) * 4>(a));
        v[1] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 8) * 4>(a));
        v[2] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 16) * 4>(a));
        v[3] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 24) * 4>(a));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
    };
    // ---- epilogues: feature n = 32 ib + 8 (r >> 2) + 4 h + (r & 3) of sample (lane, jb)
    // softplus(acc + bias) / odiv of block ib, sample block jb (the skip layer's tail: emb / u4div)
    // (x * 1 == x: the divisor's multiply only where it is not 1 -- a uniform branch, the same bits)
    auto values = [&](auto ib_c, int jb, int l, const floatx4* bb, float* o) __attribute__((always_inline)) {
        constexpr int ib = decltype(ib_c)::value;
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = softplus_hw(acc[ib][jb][r] + bb[r >> 2][r & 3], c_exp, c_thr, c_log);
        if (l == p.skip_layer) {
            const float inv_odiv = p.inv_odiv[l];
#pragma unroll
            for (int r = 0; r < 16; ++r) o[r] *= inv_odiv;
        }
    };
    // a hidden layer: its activations, RNE bf16, in the next layer's B-operand order
    auto epi_pack = [&](int l) __attribute__((always_inline)) {
        static_for<8>([&](auto ib_c) {
            constexpr int ib = decltype(ib_c)::value;
            floatx4 bb[4];
            read4(ldsBias + l * 1024, ib_c, bb);
#pragma unroll
            for (int jb = 0; jb < 2; ++jb) {
                float o[16];
                values(ib_c, jb, l, bb, o);
                // k-step 2 ib (r < 8) and 2 ib + 1 (r >= 8)
#pragma unroll
                for (int hs = 0; hs < 2; ++hs) {
                    unsigned P0 = pack_b16x2(o[8 * hs + 0], o[8 * hs + 1]);
                    unsigned P1 = pack_b16x2(o[8 * hs + 2], o[8 * hs + 3]);
                    unsigned P2 = pack_b16x2(o[8 * hs + 4], o[8 * hs + 5]);
                    unsigned P3 = pack_b16x2(o[8 * hs + 6], o[8 * hs + 7]);
                    // lower half: rows 0-3 own, 4-7 from the upper half's P0, P1; upper: 8-11 from the
                    // lower half's P2, P3, 12-15 own
                    const auto s02 = __builtin_amdgcn_permlane32_swap(P0, P2, false, false);
                    const auto s13 = __builtin_amdgcn_permlane32_swap(P1, P3, false, false);
                    const u32x4 w = {(unsigned)s02[0], (unsigned)s13[0], (unsigned)s02[1], (unsigned)s13[1]};
                    bq[jb][2 * ib + hs] = __builtin_bit_cast(bf16x8, w);
                }
            }
        });
    };
    // the skip layer: its output features n >= nout (k-steps 12 .. 15 of the next layer: nout >= 192)
    // are the tail's values -- RNE(emb / skip_div) as cn_sdf_embed writes them -- over the softplus ones,
    // per dword (feature pairs; nout % 4 == 0).  Lane half h of k-step ks holds features 16 ks + 8 h + j.
    auto fix_tail = [&](int l) __attribute__((always_inline)) {
        const int nout = p.nout[l];
        u32x4 t[2][4];
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            const int m = blk * 256 + wave * 64 + 32 * jb + l31;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // the group straddling nout starts at column -4 (nout % 4 == 0): load from column 0 and move
                // the first two dwords up to the features >= nout
                const int c0 = 16 * (12 + k) + 8 * h - nout;
                const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(vt, (m * p.ld_t + max(c0, 0)) * 2, 0, 0);
                t[jb][k] = c0 < 0 ? u32x4{w[0], w[1], w[0], w[1]} : w;
            }
        }
        wait_vmcnt<0>();  // (a drain: the ring's chunks in flight land too; once per block)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u32x4 w = __builtin_bit_cast(u32x4, bq[jb][12 + k]);
#pragma unroll
                for (int d = 0; d < 4; ++d) w[d] = 16 * (12 + k) + 8 * h + 2 * d >= nout ? t[jb][k][d] : w[d];
                bq[jb][12 + k] = __builtin_bit_cast(bf16x8, w);
            }
    };
    // the head: the DMA tile's row-dot order -- per sample, column half wn = ib >> 2 and column lane
    // lcol = (r & 3) + 8 (r >> 2) + 4 h: Σ over the column blocks j = ib & 3 in order, then the 32-lane
    // butterfly over lcol (offsets 16, 8, 4, 2, 1: r ^ 8, r ^ 4, the other half, r ^ 2, r ^ 1), then
    // the halves in order, then the bias
    auto epi_head = [&]() __attribute__((always_inline)) {
        constexpr int l = kMlpLayers - 1;
        const float hb = p.head_b[0];
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {  // one sample block at a time (32 partials live, not 64)
            float part[2][16];
            static_for<8>([&](auto ib_c) {
                constexpr int ib = decltype(ib_c)::value;
                floatx4 bb[4], hw[4];
                read4(ldsBias + l * 1024, ib_c, bb);
                read4(ldsHead, ib_c, hw);
                float o[16];
                values(ib_c, jb, l, bb, o);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float x = o[r] * hw[r >> 2][r & 3];
                    part[ib >> 2][r] = (ib & 3) == 0 ? 0.0f + x : part[ib >> 2][r] + x;
                }
            });
            float sw2[2];
#pragma unroll
            for (int wn = 0; wn < 2; ++wn) {
                float t1[8], t2[4], t3[4];
#pragma unroll
                for (int r = 0; r < 8; ++r) t1[r] = part[wn][r] + part[wn][r ^ 8];
#pragma unroll
                for (int r = 0; r < 4; ++r) t2[r] = t1[r] + t1[r ^ 4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const unsigned u = __builtin_bit_cast(unsigned, t2[r]);
                    const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
                    t3[r] = __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
                }
                const float t4a = t3[0] + t3[2], t4b = t3[1] + t3[3];
                sw2[wn] = t4a + t4b;
            }
            const int row = blk * 256 + wave * 64 + 32 * jb + l31;
            if (h == 0 && row < p.M) p.sdf[p.idx ? is[jb] : row] = (sw2[0] + sw2[1]) + hb;
        }
    };

    for (; blk < p.nblocks; blk += gridDim.x) {
        // lin0's input: the embedding's bf16 image, k = 16 ks + 8 h + j; the sdf destinations.  (A
        // drain: the ring's chunks in flight land too -- one wait per block)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            const int m = blk * 256 + wave * 64 + 32 * jb + l31;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                bq[jb][ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(vu, (m * p.ld_u0 + 16 * ks + 8 * h) * 2, 0, 0));
            is[jb] = __builtin_amdgcn_raw_buffer_load_b32(vi, m * 4, 0, 0);
        }
        wait_vmcnt<0>();
        dump(0, 4);
        zero_acc();
        static_for<2>(chunk);
        epi_pack(0);
        dump(1, 16);
        for (int l = 1; l < kMlpLayers - 1; ++l) {
            zero_acc();
            static_for<8>(chunk);
            epi_pack(l);
            if (l == p.skip_layer) fix_tail(l);
            dump(l + 1, 16);
        }
        // lin7 and the head (peeled: the chain's input registers are dead in the head's epilogue)
        zero_acc();
        static_for<8>(chunk);
        epi_head();
    }
    wait_vmcnt<0>();  // the ring's last chunks land before the workgroup ends
}


// ---------------------------------------------------------------------------------------------------------
// The same query in the fp32-class bf16x6 mode (config C2's GEMMs: every fp32 operand three RNE bf16 terms,
// the six products with i + j <= 2, fp32 accumulate; cn_gemm.hip MODE 2).  One persistent workgroup of
// four waves per CU takes 128 samples at a time (wave w: samples 32 w + (lane & 31)) through lin0 .. lin7
// and the sdf row:
//
//  * the activations stay in registers as fp32 in the B-operand order (lane half h: features 16 ks + 8 h
//    .. + 7 of k-step ks; 128 VGPRs for 32 samples x 256 features) and are split into their three terms per
//    k-step, beside the MFMAs (the layer path splits them while staging: the same split3, the same bits);
//    after a layer's epilogue (bias, softplus) four v_permlane32_swap per 8 values reorder the accumulator
//    layout into the next layer's operand order;
//  * the weights stream through an LDS-DMA ring of one 16-deep k-step per slot: that k-step's chunk of the
//    layer's chunk-major term image ([256 rows][3 terms][16], 24 KB, contiguous in HBM / L2), 6 slots,
//    5 in flight across layer and block boundaries; four waves share every byte fetched;
//  * products are issued per output block in the layer path's order (k-steps ascending; per k-step the
//    term pairs (act, weight) = (0,0) (1,0) (0,1) (2,0) (1,1) (0,2)), operands swapped (outᵀ = W · actᵀ),
//    so every activation is bitwise the layer path's (cn_linear on the 128x128 tile for lin0, the
//    256x256 tiles after, SOFTPLUS_HEAD's row-dot order for the sdf).
// Per sample: the embedding's fp32 rows in (lin0's input, 256 B; the skip tail, 4 E B), the sdf out.
#ifndef CN_X6Q_EXP
#define CN_X6Q_EXP 0  // measurement builds: 1 no weight stream, 2 no softplus in the epilogue
#endif
#ifndef CN_X6Q_SPLIT_AHEAD
#define CN_X6Q_SPLIT_AHEAD 1
#endif
#ifndef CN_X6Q_DMA
#define CN_X6Q_DMA 1  // 0: register staging of the weight chunks (measured 6 % slower, profiles/r6_ab.txt r6h)
#endif
constexpr int kX6NS = CN_X6Q_DMA ? 6 : 3;  // ring slots
constexpr int kX6Chunk = 24576;     // bytes per slot: 256 rows x 3 terms x 16 k bf16
constexpr int kX6StepsPerBlock = 4 + 7 * 16;  // k-steps of lin0 (K = 64) and lin1 .. lin7 (K = 256)

struct SdfMlpX6Args {
    const float* u0;                  // [M][ld_u0] fp32: the embedding, 64 columns (lin0's input)
    const float* tail;                // [M][ld_t] fp32: the embedding / u4div (the skip layer's tail)
    int ld_u0, ld_t, M, nblocks;
    const bf16_t* W[kMlpLayers];      // chunk-major term images [K/16][256 rows][48]
    const float* bias[kMlpLayers];
    int nout[kMlpLayers];
    float inv_odiv[kMlpLayers];
    const float* head_w;              // [256] sdf row of lin8 / scale
    const float* head_b;
    float* sdf;
    const int* idx;
    int skip_layer;
    float beta, threshold;
    float* dbg;                       // (DBG) every layer's input, fp32 [8][M][256]
};

template <bool DBG>
__global__ void __launch_bounds__(256, 1) sdf_mlp_x6_kernel(SdfMlpX6Args p) {
    __shared__ __attribute__((aligned(16))) char smem[kX6NS * kX6Chunk + kMlpLayers * 256 * 4 + 256 * 4];
    float* sBias = reinterpret_cast<float*>(smem + kX6NS * kX6Chunk);
    float* sHead = sBias + kMlpLayers * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l31 = lane & 31;

    for (int i = tid; i < kMlpLayers * 256; i += 256) {
        const int l = i >> 8, n = i & 255;
        sBias[i] = n < p.nout[l] ? p.bias[l][n] : 0.0f;
    }
    sHead[tid] = p.head_w[tid];
    __syncthreads();

    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
    const uint32_t ldsBias = lds0 + kX6NS * kX6Chunk;
    const uint32_t ldsHead = ldsBias + kMlpLayers * 256 * 4;

    // The slot's rows are 96 bytes (24 dwords): rows r and r + 8 would start on the same bank quad, a two-way
    // conflict in every ds_read_b128 lane group.  So the six 16-byte pieces of a row with (r >> 3) odd are
    // rotated by one place (its data starts 4 banks over): the fragment reads are conflict-free.  The DMA
    // writes LDS linearly, so the rotation is in each lane's source offset: physical piece pp of the slot
    // (= 384 w + 64 j + lane) holds logical piece (pp % 6 - rot(pp / 6)) mod 6 of row pp / 6.
    int dvo[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int pp = wave * 384 + j * 64 + lane, row = pp / 6;
        dvo[j] = row * 96 + ((pp % 6 + 6 - ((row >> 3) & 1)) % 6) * 16;
    }
    // k-step g of the workgroup's stream: step g % 116 of a sample block -> (layer, chunk)
    auto step_of = [](int sb, int& l, int& c) __attribute__((always_inline)) {
        if (sb < 4) {
            l = 0;
            c = sb;
        } else {
            l = 1 + ((sb - 4) >> 4);
            c = (sb - 4) & 15;
        }
    };
    // wave w copies bytes 6 KB w .. + 6 KB of the slot: six 1 KB pieces, lane l -> 16 bytes at 16 l (the LDS
    // image is the chunk as it lies in the term image: row r at 96 r, term t at + 32 t, k half h at + 16 h)
    auto chunk_view = [&](int g) __attribute__((always_inline)) {
        int l, c;
        step_of(g % kX6StepsPerBlock, l, c);
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.W[l]) + (int64_t)c * 256 * 48, 0, kX6Chunk,
                                                 0x00020000);
    };
    auto issue = [&](int g) __attribute__((always_inline)) {
        if (CN_X6Q_EXP == 1 || !CN_X6Q_DMA) return;  // (measurement build: no weight stream)
        const rsrc_t v = chunk_view(g);
        char* dst = smem + (g % kX6NS) * kX6Chunk + wave * 6144;
#pragma unroll
        for (int j = 0; j < 6; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(v, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16,
                                                     dvo[j], 0, 0, 0);
    };
    // Register staging (CN_X6Q_DMA 0): a chunk's 6 pieces per lane are loaded one k-step ahead and written to their
    // slot positions by ds_write_b128 -- about a sixth of an LDS-DMA piece's issue cycles each
    floatx4 stg[6];
    auto gload = [&](int g) __attribute__((always_inline)) {
        if (CN_X6Q_EXP == 1 || CN_X6Q_DMA) return;
        const rsrc_t v = chunk_view(g);
#pragma unroll
        for (int j = 0; j < 6; ++j) stg[j] = bload4(v, dvo[j], 0);
    };
    auto swrite = [&](int g) __attribute__((always_inline)) {
        if (CN_X6Q_EXP == 1 || CN_X6Q_DMA) return;
        wait_vmcnt<0>();
        char* dst = smem + (g % kX6NS) * kX6Chunk + wave * 6144 + lane * 16;
#pragma unroll
        for (int j = 0; j < 6; ++j) *reinterpret_cast<floatx4*>(dst + j * 1024) = stg[j];
    };
    // weight (A operand) reads: lane l -> row (l & 31) of 32-row block ib (32 rows keep the rotation), term t,
    // k half h: logical piece 2 t + h
    uint32_t aoff[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) aoff[t] = l31 * 96 + ((2 * t + h + ((l31 >> 3) & 1)) % 6) * 16;

    const float c_exp = p.beta * 1.44269504088896341f;
    const float c_thr = p.threshold * 1.44269504088896341f;
    const float c_log = 0.693147180559945309f / p.beta;

    const rsrc_t vu = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.u0), 0, p.M * p.ld_u0 * 4, 0x00020000);
    const rsrc_t vt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.tail), 0, p.M * p.ld_t * 4, 0x00020000);
    const rsrc_t vi = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.idx), 0, p.idx ? p.M * 4 : 0, 0x00020000);
    int isd = 0;

    int blk = blockIdx.x;
    if (blk >= p.nblocks) return;
    int g = 0;
#pragma unroll
    for (int d = 0; d < kX6NS - 2; ++d) issue(d);
    if constexpr (!CN_X6Q_DMA) {  // chunks 0, 1 in their slots, chunk 2 in the staging registers
        gload(0);
        swrite(0);
        gload(1);
        swrite(1);
        gload(2);
    }

    floatx4 act[16][2];  // the current layer's input: k-step ks, lane half h: features 16 ks + 8 h + 4 e + (0..3)
    floatx16 acc[8];
    auto dump = [&](int l, int nks) __attribute__((always_inline)) {
        if constexpr (DBG) {
            const int m = blk * 128 + wave * 32 + l31;
            if (m < p.M)
#pragma unroll
                for (int ks = 0; ks < 16; ++ks)
                    if (ks < nks)
#pragma unroll
                        for (int e = 0; e < 2; ++e)
                            *reinterpret_cast<floatx4*>(p.dbg + ((int64_t)l * p.M + m) * 256 + 16 * ks + 8 * h + 4 * e) =
                                act[ks][e];
        }
    };
    // one 16-deep k-step (stream position g) of the layer: the activations' terms, then per output block
    // the six products in the layer path's order
    // weight terms 0 and 1 of the current k-step's eight blocks: read at the end of the previous k-step (its
    // last products then run beside those reads), term 2 mid-step
    bf16x8 w0[8], w1[8];
    auto read_w = [&](int gg, auto t_c) __attribute__((always_inline)) {
        constexpr int t = decltype(t_c)::value;
        const uint32_t sb = lds0 + (gg % kX6NS) * kX6Chunk + aoff[t];
        static_for<8>([&](auto ib_c) {
            constexpr int ib = decltype(ib_c)::value;
            const bf16x8 v = __builtin_bit_cast(bf16x8, lds_read_b128<ib * 32 * 96>(sb));
            if constexpr (t == 0) w0[ib] = v;
            else w1[ib] = v;
        });
    };
    // k-step g's chunk certified landed by every wave (this wave's pieces: the NS - 3 later chunks may fly;
    // the barrier: every wave's, and every wave done reading chunk g - 2's slot, which the DMA issued here
    // refills with chunk g + NS - 2)
    // (register staging: the barrier certifies chunk g written by every wave a step earlier -- each wave's
    // writes retired by the lgkmcnt(0) -- and every wave done with chunk g - 2's slot)
    auto land = [&](int gg) __attribute__((always_inline)) {
        if constexpr (CN_X6Q_DMA) {
            wait_vmcnt<6 * (kX6NS - 3)>();
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(gg + kX6NS - 2);
    };
    // one 16-deep k-step (stream position g) of the layer: the activations' terms, then per output block the
    // six products in the layer path's order; chunk g + 1 is certified and its terms 0, 1 read before the
    // sixth product
    // the three terms of k-step ks's activations (the layer path splits them while staging: the same split3)
    auto split_act = [&](int ks, bf16x8& b0, bf16x8& b1, bf16x8& b2) __attribute__((always_inline)) {
        bf16x4 a0[2], a1[2], a2[2];
        split3(act[ks][0], a0[0], a1[0], a2[0]);
        split3(act[ks][1], a0[1], a1[1], a2[1]);
        b0 = __builtin_shufflevector(a0[0], a0[1], 0, 1, 2, 3, 4, 5, 6, 7);
        b1 = __builtin_shufflevector(a1[0], a1[1], 0, 1, 2, 3, 4, 5, 6, 7);
        b2 = __builtin_shufflevector(a2[0], a2[1], 0, 1, 2, 3, 4, 5, 6, 7);
    };
    bf16x8 nb0, nb1, nb2;  // (CN_X6Q_SPLIT_AHEAD) the next k-step's terms, split beside this step's products
    auto kstep_n = [&](auto ks_c, auto nks_c) __attribute__((always_inline)) {
        constexpr int ks = decltype(ks_c)::value, NKS = decltype(nks_c)::value;
        const uint32_t sb = lds0 + (g % kX6NS) * kX6Chunk + aoff[2];
        bf16x8 b0, b1, b2;
        if (CN_X6Q_SPLIT_AHEAD && ks > 0) {
            b0 = nb0;
            b1 = nb1;
            b2 = nb2;
        } else {
            split_act(ks, b0, b1, b2);
        }
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(w0[0]), "+v"(w0[1]), "+v"(w0[2]), "+v"(w0[3]), "+v"(w0[4]),
                     "+v"(w0[5]), "+v"(w0[6]), "+v"(w0[7]));
        // (act term, weight term) = (0,0), (1,0) on every block
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0[ib], b0, acc[ib], 0, 0, 0);
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0[ib], b1, acc[ib], 0, 0, 0);
        if constexpr (CN_X6Q_SPLIT_AHEAD && ks + 1 < NKS) split_act(ks + 1, nb0, nb1, nb2);
        bf16x8 w2[8];
        static_for<8>([&](auto ib_c) {
            constexpr int ib = decltype(ib_c)::value;
            w2[ib] = __builtin_bit_cast(bf16x8, lds_read_b128<ib * 32 * 96>(sb));
        });
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(w1[0]), "+v"(w1[1]), "+v"(w1[2]), "+v"(w1[3]), "+v"(w1[4]),
                     "+v"(w1[5]), "+v"(w1[6]), "+v"(w1[7]));
        // (0,1), (2,0), (1,1)
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1[ib], b0, acc[ib], 0, 0, 0);
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0[ib], b2, acc[ib], 0, 0, 0);
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1[ib], b1, acc[ib], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        swrite(g + 2);  // (register staging) chunk g + 2, loaded a step ago, into chunk g - 1's slot
        gload(g + 3);
        land(g + 1);
        read_w(g + 1, std::integral_constant<int, 0>{});
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(w2[0]), "+v"(w2[1]), "+v"(w2[2]), "+v"(w2[3]), "+v"(w2[4]),
                     "+v"(w2[5]), "+v"(w2[6]), "+v"(w2[7]));
        // (0,2), beside the next chunk's term-1 reads
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2[ib], b0, acc[ib], 0, 0, 0);
        read_w(g + 1, std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
        ++g;
    };
    auto kstep4 = [&](auto ks_c) __attribute__((always_inline)) { kstep_n(ks_c, std::integral_constant<int, 4>{}); };
    auto kstep = [&](auto ks_c) __attribute__((always_inline)) { kstep_n(ks_c, std::integral_constant<int, 16>{}); };
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int ib = 0; ib < 8; ++ib)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[ib][r] = 0.0f;
    };
    auto read4 = [&](uint32_t base, auto ib_c, floatx4* v) __attribute__((always_inline)) {
        constexpr int ib = decltype(ib_c)::value;
        const uint32_t a = base + 16 * h;
        v[0] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 0) * 4>(a));
        v[1] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 8) * 4>(a));
        v[2] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 16) * 4>(a));
        v[3] = __builtin_bit_cast(floatx4, lds_read_b128<(32 * ib + 24) * 4>(a));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
    };
    // feature n = 32 ib + 8 (r >> 2) + 4 h + (r & 3): softplus(acc + bias) / odiv, as cn_linear's epilogue
    auto values = [&](auto ib_c, int l, const floatx4* bb, float* o) __attribute__((always_inline)) {
        constexpr int ib = decltype(ib_c)::value;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            o[r] = CN_X6Q_EXP == 2 ? acc[ib][r] + bb[r >> 2][r & 3]  // (measurement build: no softplus)
                                   : softplus_hw(acc[ib][r] + bb[r >> 2][r & 3], c_exp, c_thr, c_log);
        if (l == p.skip_layer) {
            const float inv_odiv = p.inv_odiv[l];
#pragma unroll
            for (int r = 0; r < 16; ++r) o[r] *= inv_odiv;
        }
    };
    // a hidden layer's activations in the next layer's operand order: k-steps 2 ib (r < 8) and 2 ib + 1;
    // lane half 0 keeps its rows r .. r + 3 and takes the other half's, half 1 the reverse with r + 4 .. r + 7
    auto epi_act = [&](int l) __attribute__((always_inline)) {
        static_for<8>([&](auto ib_c) {
            constexpr int ib = decltype(ib_c)::value;
            floatx4 bb[4];
            read4(ldsBias + l * 1024, ib_c, bb);
            float o[16];
            values(ib_c, l, bb, o);
#pragma unroll
            for (int hs = 0; hs < 2; ++hs) {
                float lo[4], hi[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, o[8 * hs + d]),
                                                                     __builtin_bit_cast(unsigned, o[8 * hs + 4 + d]),
                                                                     false, false);
                    lo[d] = __builtin_bit_cast(float, (unsigned)sw[0]);
                    hi[d] = __builtin_bit_cast(float, (unsigned)sw[1]);
                }
                act[2 * ib + hs][0] = floatx4{lo[0], lo[1], lo[2], lo[3]};
                act[2 * ib + hs][1] = floatx4{hi[0], hi[1], hi[2], hi[3]};
            }
        });
    };
    // the skip layer: features n >= nout are the tail's fp32 values (emb / skip_div as cn_sdf_embed writes
    // them), k-steps 12 .. 15 (nout >= 192)
    auto fix_tail = [&](int l) __attribute__((always_inline)) {
        const int nout = p.nout[l];
        const int m = blk * 128 + wave * 32 + l31;
        float t[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = 16 * (12 + k) + 8 * h + j - nout;
                t[k][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vt, (m * p.ld_t + max(c, 0)) * 4, 0, 0));
            }
        wait_vmcnt<0>();  // (a drain, once per block: the ring's chunks in flight land too)
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                floatx4 v = act[12 + k][e];
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = 16 * (12 + k) + 8 * h + 4 * e + q >= nout ? t[k][4 * e + q] : v[q];
                act[12 + k][e] = v;
            }
    };
    // the head: cn_linear SOFTPLUS_HEAD's row-dot order on the 64x128 wave tiles (cn_sdf_mlp's epi_head)
    auto epi_head = [&]() __attribute__((always_inline)) {
        constexpr int l = kMlpLayers - 1;
        const float hb = p.head_b[0];
        float part[2][16];
        static_for<8>([&](auto ib_c) {
            constexpr int ib = decltype(ib_c)::value;
            floatx4 bb[4], hw[4];
            read4(ldsBias + l * 1024, ib_c, bb);
            read4(ldsHead, ib_c, hw);
            float o[16];
            values(ib_c, l, bb, o);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float x = o[r] * hw[r >> 2][r & 3];
                part[ib >> 2][r] = (ib & 3) == 0 ? 0.0f + x : part[ib >> 2][r] + x;
            }
        });
        float sw2[2];
#pragma unroll
        for (int wn = 0; wn < 2; ++wn) {
            float t1[8], t2[4], t3[4];
#pragma unroll
            for (int r = 0; r < 8; ++r) t1[r] = part[wn][r] + part[wn][r ^ 8];
#pragma unroll
            for (int r = 0; r < 4; ++r) t2[r] = t1[r] + t1[r ^ 4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned u = __builtin_bit_cast(unsigned, t2[r]);
                const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
                t3[r] = __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
            }
            const float t4a = t3[0] + t3[2], t4b = t3[1] + t3[3];
            sw2[wn] = t4a + t4b;
        }
        const int row = blk * 128 + wave * 32 + l31;
        if (h == 0 && row < p.M) p.sdf[p.idx ? isd : row] = (sw2[0] + sw2[1]) + hb;
    };

    // the prefetched fragments complete (and become values the compiler may move) before any control-flow
    // merge: a layer's end, the layer and block loops' back edges (a register copy the compiler inserts there
    // would copy a read still in flight)
    auto settle_w = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w0[0]), "+v"(w0[1]), "+v"(w0[2]), "+v"(w0[3]), "+v"(w0[4]),
                     "+v"(w0[5]), "+v"(w0[6]), "+v"(w0[7]));
        asm volatile("" : "+v"(w1[0]), "+v"(w1[1]), "+v"(w1[2]), "+v"(w1[3]), "+v"(w1[4]), "+v"(w1[5]), "+v"(w1[6]),
                     "+v"(w1[7]));
    };
    land(0);
    read_w(0, std::integral_constant<int, 0>{});
    read_w(0, std::integral_constant<int, 1>{});
    settle_w();
    for (; blk < p.nblocks; blk += gridDim.x) {
        {
            const int m = blk * 128 + wave * 32 + l31;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                for (int e = 0; e < 2; ++e)
                    act[ks][e] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 vu, (m * p.ld_u0 + 16 * ks + 8 * h + 4 * e) * 4, 0, 0));
            isd = __builtin_amdgcn_raw_buffer_load_b32(vi, m * 4, 0, 0);
        }
        wait_vmcnt<0>();
        dump(0, 4);
        zero_acc();
        static_for<4>(kstep4);
        settle_w();
        epi_act(0);
        dump(1, 16);
        for (int l = 1; l < kMlpLayers - 1; ++l) {
            zero_acc();
            static_for<16>(kstep);
            settle_w();
            epi_act(l);
            if (l == p.skip_layer) fix_tail(l);
            dump(l + 1, 16);
        }
        zero_acc();
        static_for<16>(kstep);
        settle_w();
        epi_head();
    }
    wait_vmcnt<0>();
}


}  // namespace cn

using namespace cn;

static int sdf_mlp_x6(const cn_sdf_mlp_desc* d, cn_stream_t stream) {
    const int E = 4 * (1 + 2 * d->multires);
    CN_REQUIRE(d->ld_u0 >= 64 && d->ld_u0 % 4 == 0 && al16(d->u0) && d->ld_t >= E && ((uintptr_t)d->tail & 3) == 0,
               CN_ERR_ALIGN, "cn_sdf_mlp (bf16x6): u0 fp32 [M][64] (ld %% 4, 16-byte aligned) / tail fp32 [M][E]");
    CN_REQUIRE((int64_t)d->M * (d->ld_u0 > d->ld_t ? d->ld_u0 : d->ld_t) * 4 < ((int64_t)1 << 31), CN_ERR_SHAPE,
               "cn_sdf_mlp: M = %d too large for one launch", d->M);
    SdfMlpX6Args a{};
    for (int l = 0; l < kMlpLayers; ++l) {
        CN_REQUIRE(d->W[l] && d->bias[l] && d->ldw[l] == 256 && al16(d->W[l]), CN_ERR_ARG,
                   "cn_sdf_mlp (bf16x6): layer %d needs a chunk-major term image of 256 rows (ldw %lld)", l,
                   (long long)d->ldw[l]);
        a.W[l] = static_cast<const bf16_t*>(d->W[l]);
        a.bias[l] = d->bias[l];
        a.nout[l] = l == d->skip_layer ? 256 - E : 256;
        a.inv_odiv[l] = l == d->skip_layer ? 1.0f / d->skip_div : 1.0f;
    }
    a.u0 = static_cast<const float*>(d->u0);
    a.tail = static_cast<const float*>(d->tail);
    a.ld_u0 = (int)d->ld_u0;
    a.ld_t = (int)d->ld_t;
    a.M = d->M;
    a.nblocks = (d->M + 127) / 128;
    a.head_w = d->head_w;
    a.head_b = d->head_b;
    a.sdf = d->sdf;
    a.idx = d->idx;
    a.skip_layer = d->skip_layer;
    a.beta = d->beta;
    a.threshold = d->threshold;
    if (d->M == 0) return CN_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const int grid = a.nblocks < cus ? a.nblocks : cus;
    a.dbg = static_cast<float*>(d->debug);
    if (a.dbg)
        sdf_mlp_x6_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    else
        sdf_mlp_x6_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    return check_launch("cn_sdf_mlp");
}

extern "C" int cn_sdf_mlp(const cn_sdf_mlp_desc* d, cn_stream_t stream) {
    CN_REQUIRE(d && d->u0 && d->tail && d->sdf && d->head_w && d->head_b, CN_ERR_ARG, "cn_sdf_mlp: null pointer");
    CN_REQUIRE(d->format == 0 || d->format == CN_MFMA_F32_BF16X6, CN_ERR_UNSUPPORTED,
               "cn_sdf_mlp: format %d (0: bf16 images, CN_MFMA_F32_BF16X6: fp32 inputs and term images)", d->format);
    if (d->format == CN_MFMA_F32_BF16X6) {
        CN_REQUIRE(d->n_layers == kMlpLayers && d->hidden == 256 && d->kpad0 == 64, CN_ERR_UNSUPPORTED,
                   "cn_sdf_mlp: %d layers of width %d (first K %d); the fused query takes 8 x 256 (K0 = 64)",
                   d->n_layers, d->hidden, d->kpad0);
        CN_REQUIRE(d->multires >= 0 && 4 * (1 + 2 * d->multires) <= 64 && d->skip_layer >= 1 &&
                       d->skip_layer < kMlpLayers - 1 && 256 - 4 * (1 + 2 * d->multires) >= 192,
                   CN_ERR_UNSUPPORTED, "cn_sdf_mlp: multires %d / skip layer %d", d->multires, d->skip_layer);
        CN_REQUIRE(d->M >= 0, CN_ERR_SHAPE, "cn_sdf_mlp: M = %d", d->M);
        return sdf_mlp_x6(d, stream);
    }
    CN_REQUIRE(d->n_layers == kMlpLayers && d->hidden == 256 && d->kpad0 == 64, CN_ERR_UNSUPPORTED,
               "cn_sdf_mlp: %d layers of width %d (first K %d); the fused query takes 8 x 256 (K0 = 64)",
               d->n_layers, d->hidden, d->kpad0);
    const int E = 4 * (1 + 2 * d->multires);
    CN_REQUIRE(d->multires >= 0 && E <= 64 && d->skip_layer >= 1 && d->skip_layer < kMlpLayers - 1, CN_ERR_UNSUPPORTED,
               "cn_sdf_mlp: multires %d / skip layer %d", d->multires, d->skip_layer);
    CN_REQUIRE(d->M >= 0 && d->ld_u0 >= 64 && d->ld_u0 % 8 == 0 && al16(d->u0) && d->ld_t >= E && d->ld_t % 4 == 0 &&
                   ((uintptr_t)d->tail & 7) == 0,
               CN_ERR_ALIGN, "cn_sdf_mlp: u0 [M][64] (ld %% 8, 16-byte aligned) / tail [M][E] (ld %% 4, 8-byte aligned)");
    CN_REQUIRE((int64_t)d->M * (d->ld_u0 > d->ld_t ? d->ld_u0 : d->ld_t) * 2 < ((int64_t)1 << 31), CN_ERR_SHAPE,
               "cn_sdf_mlp: M = %d too large for one launch", d->M);
    SdfMlpArgs a{};
    for (int l = 0; l < kMlpLayers; ++l) {
        const int K = l == 0 ? 64 : 256;
        const int nout = l == d->skip_layer ? 256 - E : 256;
        CN_REQUIRE(d->W[l] && d->bias[l] && d->ldw[l] >= K && d->ldw[l] % 8 == 0 && al16(d->W[l]), CN_ERR_ARG,
                   "cn_sdf_mlp: layer %d weights [256][%d] (ld %lld)", l, K, (long long)d->ldw[l]);
        a.W[l] = static_cast<const bf16_t*>(d->W[l]);
        a.ldw[l] = (int)d->ldw[l];
        a.bias[l] = d->bias[l];
        a.nout[l] = nout;
        a.inv_odiv[l] = l == d->skip_layer ? 1.0f / d->skip_div : 1.0f;
    }
    a.u0 = static_cast<const bf16_t*>(d->u0);
    a.tail = static_cast<const bf16_t*>(d->tail);
    a.ld_u0 = (int)d->ld_u0;
    a.ld_t = (int)d->ld_t;
    a.M = d->M;
    a.nblocks = (d->M + 255) / 256;
    a.head_w = d->head_w;
    a.head_b = d->head_b;
    a.sdf = d->sdf;
    a.idx = d->idx;
    a.skip_layer = d->skip_layer;
    a.beta = d->beta;
    a.threshold = d->threshold;
    if (d->M == 0) return CN_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const int grid = a.nblocks < cus ? a.nblocks : cus;
    a.dbg = static_cast<bf16_t*>(d->debug);
    if (a.dbg)
        sdf_mlp_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    else
        sdf_mlp_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    return check_launch("cn_sdf_mlp");
}
