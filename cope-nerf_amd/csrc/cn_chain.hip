// cn_chain.hip — a chain of MUL layers in one kernel (gfx950, bf16 MLP mode).
//
// The ∇ₓSDF pass of SDFNetwork.gradient (model/neus_fields.py:291-303) runs the hidden layers
// backwards, s_{l-1} = (W_lᵀ s_l) ⊙ σ_{l-1}, and the first-order adjoint of the backward has the same
// form.  Layer by layer each step reads its operand image (the previous step's output), σ's
// activation image, and writes its own image: the operand re-read is a third of the traffic.  Here
// one persistent workgroup per CU takes 256 rows at a time through every step with the chained
// operand on chip, as cn_sdf_mlp does for the forward query (cn_sampler.hip):
//
//  * each wave owns 64 rows and all 256 columns: outᵀ = W_lᵀ · inᵀ with the weights as the MFMA A
//    operand (from an LDS-DMA ring of 32-deep chunks, 8 slots, 7 in flight) and the chained operand
//    as the B operand in registers; after the epilogue two v_permlane32_swap per 8 values put the
//    step's bf16 output in the next step's B-operand order;
//  * σ's activation is read straight from HBM in the accumulator layout (8-byte pieces: four
//    columns of one row per lane), two column blocks ahead of the epilogue, the first two under the
//    step's MFMAs;
//  * outputs are written from the registers: the bf16 image as 16-byte row pieces after the permlane
//    (eight consecutive columns), fp32 outputs and the split columns as 16-byte pieces of four.
//
// Bitwise equal to cn_linear's MUL on the 256x256 bf16 tile: the same MFMA over the same k order
// (operands swapped: verified equal), u = acc * (1 / adiv), σ = 1 - exp2(aux * aux_c), out = u σ with
// the split and zero columns masked to +0, RNE bf16 images.
#include "cn_mfma.h"

// measurement builds only (profiles/r5_ab.txt): no activation loads / no image stores
#ifndef CN_AB_CHAIN_NOAUX
#define CN_AB_CHAIN_NOAUX 0
#endif
#ifndef CN_AB_CHAIN_NOSTORE
#define CN_AB_CHAIN_NOSTORE 0
#endif

namespace cn {

constexpr int kChainSteps = CN_CHAIN_MAX;
constexpr int kChNS = 8;          // weight ring slots
constexpr int kChChunk = 16384;   // bytes per slot: 256 rows x 32 k bf16

struct MulChainArgs {
    const bf16_t* in;
    int ld_in, M, nblocks, n;
    const bf16_t* W[kChainSteps];
    int ldw[kChainSteps];
    const bf16_t* aux[kChainSteps];
    int ld_aux[kChainSteps];
    float aux_c[kChainSteps];
    float inv_adiv[kChainSteps];
    int nsplit[kChainSteps];
    float* split[kChainSteps];
    int ld_split[kChainSteps];
    bf16_t* out_b[kChainSteps];
    int ld_out_b[kChainSteps];
    float* out_f[kChainSteps];
    int ld_out_f[kChainSteps];
};

__global__ void __launch_bounds__(256, 1) mul_chain_kernel(MulChainArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[kChNS * kChChunk];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l31 = lane & 31;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
    const int nchunks = 8 * p.n;  // per row block: 8 chunks of 32 k per step

    // wave w fills rows 64w .. 64w + 63 of the slot: four 1 KB pieces of 16 rows; lane l -> row + (l >> 2),
    // physical 16-byte chunk l & 3 (logical chunk (l & 3) ^ ((row >> 2) & 3))
    auto issue = [&](int g) __attribute__((always_inline)) {
        const int cb = g % nchunks;
        const int t = cb >> 3, k0 = 32 * (cb & 7);
        const int ldw = p.ldw[t];
        const rsrc_t v = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.W[t]), 0, 256 * ldw * 2, 0x00020000);
        char* dst = smem + (g % kChNS) * kChChunk + wave * 64 * 64;
        const int vo = ((lane >> 2) * ldw + 8 * ((lane & 3) ^ ((lane >> 4) & 3))) * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(v, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16, vo,
                                                     ((wave * 64 + 16 * j) * ldw + k0) * 2, 0, 0);
    };
    uint32_t aoff[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) aoff[s] = l31 * 64 + (((2 * s + h) ^ ((l31 >> 2) & 3)) << 4);

    const rsrc_t vin = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.in), 0, p.M * p.ld_in * 2, 0x00020000);

    int blk = blockIdx.x;
    if (blk >= p.nblocks) return;
    int g = 0;
#pragma unroll
    for (int d = 0; d < kChNS - 1; ++d) issue(d);

    bf16x8 bq[2][16];   // the step's input, B-operand order: lane half h of k-step ks = columns 16 ks + 8 h ..
    floatx16 acc[8][2];
    u32x2 ax[3][2][4];  // σ's activation, column blocks ib % 3: [row half jb][column quad rq], 4 bf16 each

    // one 32-deep weight chunk (k-steps 2q, 2q + 1); WAIT: this wave's vector-memory operations allowed
    // after the chunk's DMA pieces (the later chunks' pieces, plus the activation loads in flight)
    auto chunk = [&](auto q_c, auto wait_c) __attribute__((always_inline)) {
        constexpr int q = decltype(q_c)::value;
        constexpr int WAIT = decltype(wait_c)::value;
        wait_vmcnt<WAIT>();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(g + kChNS - 1);
        const uint32_t sb = lds0 + (g % kChNS) * kChChunk;
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
                    acc[ib][jb] = (q == 0 && s == 0)
                                      ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ib], bq[jb][2 * q + s], floatx16{}, 0, 0, 0)
                                      : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ib], bq[jb][2 * q + s], acc[ib][jb], 0, 0, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[4]), "+v"(af[5]), "+v"(af[6]), "+v"(af[7]));
#pragma unroll
            for (int ib = 4; ib < 8; ++ib)
#pragma unroll
                for (int jb = 0; jb < 2; ++jb)
                    acc[ib][jb] = (q == 0 && s == 0)
                                      ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ib], bq[jb][2 * q + s], floatx16{}, 0, 0, 0)
                                      : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ib], bq[jb][2 * q + s], acc[ib][jb], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        ++g;
    };

    for (; blk < p.nblocks; blk += gridDim.x) {
        const int mrow = blk * 256 + wave * 64 + l31;  // + 32 jb
        // the chain's input image in B-operand order (a drain: the ring's chunks in flight land too)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
#pragma unroll
            for (int ks = 0; ks < 16; ++ks)
                bq[jb][ks] = __builtin_bit_cast(
                    bf16x8, __builtin_amdgcn_raw_buffer_load_b128(vin, ((mrow + 32 * jb) * p.ld_in + 16 * ks + 8 * h) * 2, 0, 0));
        wait_vmcnt<0>();
        for (int t = 0; t < p.n; ++t) {
            const int ld_aux = p.ld_aux[t];
            const rsrc_t vax = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.aux[t]), 0, p.M * ld_aux * 2, 0x00020000);
            // σ's activation of column block ib: columns 32 ib + 8 rq + 4 h .. + 3 of both rows
            auto load_ax = [&](auto ib_c) __attribute__((always_inline)) {
                constexpr int ib = decltype(ib_c)::value;
#pragma unroll
                for (int jb = 0; jb < 2; ++jb)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq)
#if CN_AB_CHAIN_NOAUX
                        ax[ib % 3][jb][rq] = u32x2{0x3c003c00u + (unsigned)ib, 0x3c003c00u};
#else
                        ax[ib % 3][jb][rq] = __builtin_amdgcn_raw_buffer_load_b64(
                            vax, ((mrow + 32 * jb) * ld_aux + 32 * ib + 8 * rq + 4 * h) * 2, 0, 0);
#endif
            };
            constexpr std::integral_constant<int, 4 * (kChNS - 2)> w_ring{};
            constexpr std::integral_constant<int, 4 * (kChNS - 2) + 16> w_ring_ax{};
            // chunks 0 .. 2 wait for the ring alone; the activation loads of column blocks 0 and 1 (16 per
            // lane) go out after chunk 2's pieces, so chunks 3 .. 7 allow for them
            static_for<3>([&](auto q_c) { chunk(q_c, w_ring); });
            load_ax(std::integral_constant<int, 0>{});
            load_ax(std::integral_constant<int, 1>{});
            static_for<5>([&](auto q_c) { chunk(std::integral_constant<int, 3 + decltype(q_c)::value>{}, w_ring_ax); });

            const float aux_c = p.aux_c[t], inv_adiv = p.inv_adiv[t];
            const int nsplit = p.nsplit[t];
            const int ld_split = p.ld_split[t], ld_ob = p.ld_out_b[t], ld_of = p.ld_out_f[t];
            const rsrc_t vsp = __builtin_amdgcn_make_buffer_rsrc(p.split[t], 0, p.split[t] ? p.M * ld_split * 4 : 0, 0x00020000);
            const rsrc_t vob = __builtin_amdgcn_make_buffer_rsrc(p.out_b[t], 0, p.out_b[t] ? p.M * ld_ob * 2 : 0, 0x00020000);
            const rsrc_t vof = __builtin_amdgcn_make_buffer_rsrc(p.out_f[t], 0, p.out_f[t] ? p.M * ld_of * 4 : 0, 0x00020000);
            const bool has_f = p.out_f[t] != nullptr;
            static_for<8>([&](auto ib_c) {
                constexpr int ib = decltype(ib_c)::value;
                if constexpr (ib + 2 < 8) load_ax(std::integral_constant<int, ib + 2>{});
#pragma unroll
                for (int jb = 0; jb < 2; ++jb) {
                    const int m = mrow + 32 * jb;
                    float o[16];
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const int c0 = 32 * ib + 8 * rq + 4 * h;  // this lane's 4 columns
                        const u32x2 a = ax[ib % 3][jb][rq];
                        const float act[4] = {__builtin_bit_cast(float, a[0] << 16), __builtin_bit_cast(float, a[0] & 0xffff0000u),
                                              __builtin_bit_cast(float, a[1] << 16), __builtin_bit_cast(float, a[1] & 0xffff0000u)};
                        const bool spl = c0 >= nsplit;
                        const unsigned keep = spl ? 0u : ~0u;
                        floatx4 uv;
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const float u = acc[ib][jb][4 * rq + c] * inv_adiv;
                            uv[c] = u;
                            const float v = u * sigma_from_act(act[c], aux_c);
                            o[4 * rq + c] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, v) & keep);
                        }
                        // the split columns' raw values (other lanes' stores fall past the view)
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, uv), vsp,
                                                               spl ? (m * ld_split + c0 - nsplit) * 4 : (1 << 30), 0, 0);
                        if (has_f)
                            __builtin_amdgcn_raw_buffer_store_b128(
                                __builtin_bit_cast(u32x4, floatx4{o[4 * rq], o[4 * rq + 1], o[4 * rq + 2], o[4 * rq + 3]}), vof,
                                (m * ld_of + c0) * 4, 0, 0);
                    }
                    // RNE bf16 in the next step's B-operand order, and the image
#pragma unroll
                    for (int hs = 0; hs < 2; ++hs) {
                        unsigned P0 = pack_b16x2(o[8 * hs + 0], o[8 * hs + 1]);
                        unsigned P1 = pack_b16x2(o[8 * hs + 2], o[8 * hs + 3]);
                        unsigned P2 = pack_b16x2(o[8 * hs + 4], o[8 * hs + 5]);
                        unsigned P3 = pack_b16x2(o[8 * hs + 6], o[8 * hs + 7]);
                        const auto s02 = __builtin_amdgcn_permlane32_swap(P0, P2, false, false);
                        const auto s13 = __builtin_amdgcn_permlane32_swap(P1, P3, false, false);
                        const u32x4 w = {(unsigned)s02[0], (unsigned)s13[0], (unsigned)s02[1], (unsigned)s13[1]};
                        bq[jb][2 * ib + hs] = __builtin_bit_cast(bf16x8, w);
#if !CN_AB_CHAIN_NOSTORE
                        __builtin_amdgcn_raw_buffer_store_b128(w, vob, (m * ld_ob + 16 * (2 * ib + hs) + 8 * h) * 2, 0, 0);
#endif
                    }
                }
            });
        }
    }
    wait_vmcnt<0>();  // the ring's last chunks land before the workgroup ends
}

}  // namespace cn

using namespace cn;

extern "C" int cn_mul_chain(const cn_mul_chain_desc* d, cn_stream_t stream) {
    CN_REQUIRE(d && d->src, CN_ERR_ARG, "cn_mul_chain: null descriptor / input");
    CN_REQUIRE(d->n >= 1 && d->n <= kChainSteps && d->M >= 0, CN_ERR_SHAPE, "cn_mul_chain: %d steps (1 .. %d), M = %d",
               d->n, kChainSteps, d->M);
    CN_REQUIRE(d->ld_src >= 256 && d->ld_src % 8 == 0 && al16(d->src), CN_ERR_ALIGN, "cn_mul_chain: input [M][>= 256] bf16, ld %% 8");
    int64_t maxld = d->ld_src * 2;
    MulChainArgs a{};
    for (int t = 0; t < d->n; ++t) {
        CN_REQUIRE(d->W[t] && d->aux[t], CN_ERR_ARG, "cn_mul_chain: step %d weights / activation null", t);
        CN_REQUIRE(d->ldw[t] >= 256 && d->ldw[t] % 8 == 0 && al16(d->W[t]), CN_ERR_ALIGN,
                   "cn_mul_chain: step %d weights [256][>= 256] bf16, ld %% 8", t);
        CN_REQUIRE(d->ld_aux[t] >= 256 && d->ld_aux[t] % 4 == 0 && ((uintptr_t)d->aux[t] & 7) == 0, CN_ERR_ALIGN,
                   "cn_mul_chain: step %d activation [M][>= 256] bf16, ld %% 4, 8-byte aligned", t);
        CN_REQUIRE(d->aux_beta[t] > 0.0f, CN_ERR_ARG, "cn_mul_chain: step %d needs aux_beta > 0 (sigma from aux)", t);
        CN_REQUIRE(d->nsplit[t] > 0 && d->nsplit[t] <= 256 && d->nsplit[t] % 4 == 0, CN_ERR_SHAPE,
                   "cn_mul_chain: step %d nsplit %d (a multiple of 4 in 4 .. 256)", t, d->nsplit[t]);
        CN_REQUIRE(!d->split[t] || d->nsplit[t] == 256 ||
                       (d->ld_split[t] >= 256 - d->nsplit[t] && d->ld_split[t] % 4 == 0 && al16(d->split[t])),
                   CN_ERR_ARG, "cn_mul_chain: step %d split output [M][>= %d] fp32 (ld %% 4)", t, 256 - d->nsplit[t]);
        CN_REQUIRE(d->out_b[t] || t == d->n - 1, CN_ERR_ARG, "cn_mul_chain: step %d needs its image (the next step's operand)", t);
        CN_REQUIRE(d->out_b[t] || d->out_f[t], CN_ERR_ARG, "cn_mul_chain: the last step writes nothing");
        CN_REQUIRE(!d->out_b[t] || (d->ld_out_b[t] >= 256 && d->ld_out_b[t] % 8 == 0 && al16(d->out_b[t])), CN_ERR_ALIGN,
                   "cn_mul_chain: step %d image [M][>= 256] bf16, ld %% 8", t);
        CN_REQUIRE(!d->out_f[t] || (d->ld_out_f[t] >= 256 && d->ld_out_f[t] % 4 == 0 && al16(d->out_f[t])), CN_ERR_ALIGN,
                   "cn_mul_chain: step %d fp32 output [M][>= 256], ld %% 4", t);
        a.W[t] = static_cast<const bf16_t*>(d->W[t]);
        a.ldw[t] = (int)d->ldw[t];
        a.aux[t] = static_cast<const bf16_t*>(d->aux[t]);
        a.ld_aux[t] = (int)d->ld_aux[t];
        // the constants as cn_linear derives them (linear_plan): the same bits
        a.aux_c[t] = -d->aux_beta[t] * 1.44269504088896341f;
        const float adiv = d->adiv[t] == 0.0f ? 1.0f : d->adiv[t];
        a.inv_adiv[t] = 1.0f / adiv;
        a.nsplit[t] = d->nsplit[t];
        a.split[t] = d->nsplit[t] < 256 ? d->split[t] : nullptr;
        a.ld_split[t] = (int)d->ld_split[t];
        a.out_b[t] = static_cast<bf16_t*>(d->out_b[t]);
        a.ld_out_b[t] = (int)d->ld_out_b[t];
        a.out_f[t] = d->out_f[t];
        a.ld_out_f[t] = (int)d->ld_out_f[t];
        const int64_t lds[5] = {d->ldw[t] * 2, d->ld_aux[t] * 2, d->ld_split[t] * 4, d->ld_out_b[t] * 2, d->ld_out_f[t] * 4};
        for (int64_t v : lds) maxld = v > maxld ? v : maxld;
    }
    // buffer views address rows with 32-bit byte offsets
    CN_REQUIRE((int64_t)d->M * maxld < ((int64_t)1 << 31), CN_ERR_SHAPE, "cn_mul_chain: M = %d too large for one launch", d->M);
    a.in = static_cast<const bf16_t*>(d->src);
    a.ld_in = (int)d->ld_src;
    a.M = d->M;
    a.n = d->n;
    a.nblocks = (d->M + 255) / 256;
    if (d->M == 0) return CN_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const int grid = a.nblocks < cus ? a.nblocks : cus;
    mul_chain_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a);
    return check_launch("cn_mul_chain");
}
