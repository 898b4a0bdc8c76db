// cn_gemm.hip — fp32 MFMA GEMMs for the SDF / colour MLPs (gfx950).
//
// Every Linear of SDFNetwork (model/neus_fields.py:273-283, 9 layers, Softplus
// beta=100) and RenderingNetwork (neus_fields.py:364-373, ReLU) is a GEMM over
// M = R*S sample rows with K, N <= 320.  At fp32 these layers are MFMA-bound
// (~67 FLOP per HBM byte at N=K=256 vs ~26 FLOP/B machine balance), so each
// layer is one launch of `linear_kernel`, with the bias / activation /
// derivative bookkeeping fused into the epilogue.
//
// Kernel shape (tile 0): 128x128 output tile per 256-thread workgroup, 2x2
// waves, each wave 2x2 tiles of v_mfma_f32_32x32x2_f32 (64 fp32 accumulators).
// K is streamed in 32-deep chunks through a double-buffered LDS image
// [rows][32+4] (the +4 float pad makes the ds_read_b128 fragment reads
// conflict-free).  Within a chunk, lane half h consumes k = 16h + s at MFMA
// step s, so each lane reads 4 consecutive k with one ds_read_b128.
// Tile 1 is 128x64 (4x1 waves of 1x2 tiles) for N or K = 64 shapes.
//
// The weight gradients dW = Σ_m Y[m]ᵀ X[m] are in cn_wgrad.hip.
#include "cn_mfma.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace cn {

struct LinearArgs {
    const float* A;
    const float* A2;
    const float* B;
    const float* bias;
    const float* rowv;
    const float* colv;
    const float* aux0;
    const float* aux1;
    const float* aux2;
    float* out0;
    float* out1;
    float* out_split;
    int lda, lda2, ldb, ld_aux0, ld_aux1, ld_aux2, ld_out0, ld_out1, ld_split;
    int M, N, K, K1, nzero, nsplit, n_tiles_m, n_tiles_n;
    float inv_adiv, inv_odiv, beta, threshold;
    float aux_c;       // -aux_beta * log2(e): sigma = 1 - 2^(aux_c * aux0)
    float aux2_scale;  // BWD_SOFTPLUS second-order term scale
    const float* head_w;  // SOFTPLUS_HEAD: row-dot weights [N], bias [1], output, destination rows
    const float* head_b;
    float* head_out;
    const int* head_idx;
    int flags;
    // bf16 images of the outputs (the operands of the GEMMs that consume them, rounded as their
    // staging would round them): out0 / out1 values, RNE, same columns (NULL: none)
    bf16_t* out0_b;
    bf16_t* out1_b;
    int ld_out0_b, ld_out1_b;
};


// Persistent over output tiles: gridDim.x workgroups (OCC per CU) walk the
// virtual tiles; the first K-chunk of the next tile is fetched into registers
// while the current tile's epilogue runs, so only the first tile of a
// workgroup pays the cold-start latency.
// MODE 0: A and B fp32, v_mfma_f32_32x32x2_f32, BK fp32 k per chunk.
// MODE 1: A fp32 converted to bf16 (RNE) while staging, B bf16 [N][ldb]
//         (ldb in bf16 elements), v_mfma_f32_32x32x16_bf16, BK = 64 bf16 k per
//         chunk.  The LDS image has the fp32 geometry (rows of 36 dwords:
//         conflict-free ds_read_b128 fragments).
// MODE 2: fp32 GEMM on the bf16 MFMA (CN_MFMA_F32_BF16X6).  Each fp32 operand is
//         the sum of three bf16 terms x = x0 + x1 + x2 (x0 = bf16(x), x1 =
//         bf16(x - x0), x2 = bf16(x - x0 - x1), all RNE; |x - Σ| <= 2^-27 |x|);
//         A is split while staging, B arrives split and chunk-major: chunk c
//         (k = 16c .. 16c+15) is [ldb rows][3 terms][16 k] bf16, so a tile's B
//         chunk is one contiguous 96 * BN-byte block (coalesced 16-byte pieces
//         that land on LDS rows as they are).  The six
//         products with i + j <= 2 are issued (small terms first) into one fp32
//         accumulator; the three dropped ones are below 2^-26 |a b|, under the
//         rounding of the fp32 accumulation itself.  BK = 16 k per chunk; an LDS
//         row holds the three 16-term planes (24 dwords) + 12 pad = 36 dwords,
//         the fp32 image's geometry (conflict-free fragment reads, and the C tile
//         parks in one slab).
// The accumulator layout of the two MFMAs is the same, so the epilogue is shared.
// MODE_ bit 2 (MODE 1 only): A / A2 are bf16 operand images (16-byte pieces of 8 values land on
//         the LDS rows as they are: no conversion); bit 3: BWD_RELU's aux0 / BWD_SOFTPLUS's aux1
//         and aux2 are bf16 images.
constexpr int kTblCols = 512;  // widest N with a bias / colv (the LDS column table)

#ifndef CN_DMA_A_NT
#define CN_DMA_A_NT 0  // 1: the LDS-DMA ring's A chunks loaded non-temporally (measured slower: a 32-deep chunk is half a 128-byte line; profiles/r6_ab.txt r6x)
#endif
template <int WM, int WN, int TM, int TN, int BK, int OCC, int DEPTH, int EPI, bool ROWV, int MODE_>
__global__ void __launch_bounds__(64 * WM * WN, OCC * WM * WN / 4) linear_kernel(LinearArgs p) {
    constexpr int MODE = MODE_ & 3;         // the GEMM mode (0 fp32, 1 bf16, 2 bf16x6)
    constexpr bool ABF = (MODE_ & 4) != 0;  // A, A2 bf16 images
    // MODE_ bit 3: every aux operand of the epilogue is a bf16 image (aux0: σ's activation or
    // BWD_RELU's sign source; BWD_SOFTPLUS's aux1 / aux2 too)
    constexpr bool AUX0B = (MODE_ & 8) != 0 && (EPI == CN_EPI_BWD_RELU || EPI == CN_EPI_MUL || EPI == CN_EPI_TANGENT ||
                                                EPI == CN_EPI_BWD_SOFTPLUS);
    constexpr bool AUX12B = (MODE_ & 8) != 0 && EPI == CN_EPI_BWD_SOFTPLUS;
    static_assert(!ABF || MODE == 1, "bf16 A images only in the bf16 MFMA mode");
    // MODE_ bit 4 (MODE 2, measurement build CN_AB_X6_AIMG): A arrives as a bf16x6 term image in B's chunk-major
    // format ([K/16][lda rows][3 terms][16], lda = the image's rows), staged like B: no split
    constexpr bool AX6 = (MODE_ & 16) != 0;
    static_assert(!AX6 || (MODE == 2 && BK == 16), "bf16x6 A images: 16-deep stages of the bf16x6 mode");
    constexpr int NT = 64 * WM * WN;
    const float* const cA = p.A;
    const float* const cB = p.B;
    float* const cOut0 = p.out0;
    const int cN = p.N, cNzero = p.nzero;
    const float cInvOdiv = p.inv_odiv;
    constexpr int BM = 32 * TM * WM;
    constexpr int BN = 32 * TN * WN;
    constexpr bool BF = MODE != 0;               // bf16 MFMA (modes 1, 2)
    constexpr int NPL = MODE == 2 ? 3 : 1;       // bf16 planes per operand
    // padded LDS row in dwords: 36 in every mode (BK = 32 f32 / 64 bf16 / 16 split: 3 x 8 + 12 pad)
    // (BK = 32 split: 3 x 16 + 4 pad = 52, conflict-free like wgrad_x6_kernel's rows)
    constexpr int LS = (BF ? NPL * BK / 2 : BK) + (MODE == 2 && BK == 16 ? 12 : 4);
    constexpr int EPA = ABF ? 8 : 4;             // A elements per 16-byte staging piece
    constexpr int ESA = ABF ? 2 : 4;             // bytes per A element
    constexpr int KC4 = BK / EPA;                // A: 16-byte pieces per staged row
    static_assert(NT % KC4 == 0, "staging rows");
    constexpr int RSTEP = NT / KC4;  // staged A rows per load instruction
    constexpr int KCB = BF ? NPL * BK / 8 : BK / 4;  // B: 16-byte pieces per staged row (all planes)
    // modes 0/1: B rows tid/KCB + q*RSTEPB; mode 2 (6 pieces per row): piece tid + q*NT
    constexpr int RSTEPB = MODE == 2 ? 1 : NT / KCB;
    static_assert(BM % RSTEP == 0 && (MODE == 2 || (NT % KCB == 0 && BN % RSTEPB == 0)), "tile/thread mismatch");
    constexpr int ALD = AX6 ? (BM * 6 + NT - 1) / NT : BM / RSTEP;  // (AX6: 16-byte pieces like B's)
    constexpr int BLD = MODE == 2 ? (BN * KCB + NT - 1) / NT : BN / RSTEPB;
    constexpr int ESZB = BF ? 2 : 4;             // bytes per B element
    constexpr int PIECES_PL = BK / 8;            // MODE 2: 16-byte pieces per plane of a staged row
    constexpr int CS = BN + 4;
    constexpr int LDS_FLOATS = 2 * BM * LS + 2 * BN * LS;
    // the epilogue parks the C tile in the staging LDS, in NPART row slabs if it does not fit
    constexpr int NPART = (BM * CS <= LDS_FLOATS) ? 1 : ((BM / 2) * CS <= LDS_FLOATS ? 2 : 4);
    static_assert((BM / NPART) * CS <= LDS_FLOATS, "C tile slab must fit in the staging LDS");
    constexpr int PROWS = BM / NPART;

    // bias / colv of every column (N <= kTblCols, host-checked) live in LDS past the staging
    // buffers, filled once per workgroup: the epilogue issues no vector-memory load for them,
    // so its only VMEM waits are for the aux rows it reads (the compiler's vmcnt for a
    // per-tile bias load, under the divergent region branch, was a full drain before every
    // pass -- each pass waited for the previous pass's stores)
    // (SOFTPLUS_HEAD: + the head weights and bias; its rows fit one tile, N <= 256)
    constexpr bool kHead = EPI == CN_EPI_SOFTPLUS_HEAD;
    constexpr bool kBias = EPI == CN_EPI_STORE || EPI == CN_EPI_SOFTPLUS || EPI == CN_EPI_RELU || kHead;
    constexpr bool kColv = ROWV || kHead;
    constexpr int TBLC = kHead ? 256 : kTblCols;
    constexpr int TBL = (kBias ? TBLC : 0) + (kColv ? TBLC : 0) + (kHead ? TBLC + 4 : 0);
    // The 256x256 bf16 tile with bf16 A images stages A and B by LDS-DMA into a ring of DNS stages
    // (no register staging: DNS - 1 = 3 stages, 96 KB, in flight per CU, across tile boundaries,
    // under the epilogue too).  A stage is the BM A rows and BN B rows of one 32-deep chunk, 64-byte
    // rows whose 16-byte chunks are XOR-swizzled by (row >> 2) & 3 (the DMA writes LDS linearly, the
    // swizzle is in the per-lane global address): the ds_read_b128 lane groups of the MFMA operand
    // reads ({0-3, 12-15, 20-27}, ...) then hit 16 distinct bank quads.  + 2 * BM floats: the
    // SOFTPLUS_HEAD row partials (the ring is busy with the next tile's stages during the epilogue).
    constexpr bool kDma = ABF && MODE == 1 && TM * TN >= 8 && BK == 32 && OCC == 1 && BM == 256 && BN == 256;
    constexpr int DNS = 4, DROWB = BK * 2, DSIDEA = BM * DROWB, DSTAGE = (BM + BN) * DROWB;
    constexpr int LDS_MAIN = kDma ? DNS * DSTAGE / 4 + 2 * BM : LDS_FLOATS;
    __shared__ __attribute__((aligned(16))) float smem[LDS_MAIN + TBL];
    float* sA = smem;
    float* sB = smem + 2 * BM * LS;
    float* sBias = smem + LDS_MAIN;
    float* sColv = sBias + (kBias ? TBLC : 0);
    float* sHeadW = sColv + (kColv ? TBLC : 0);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;
    const int T = p.n_tiles_n;
    const int ntiles = ((p.n_tiles_m + 7) / 8) * 8 * T;
    const int nk = p.K / BK;

    // staging: thread tid loads A rows tid/KC4 + q*RSTEP (16-byte piece tid%KC4: 4 fp32 or 8 bf16)
    // and B rows tid/KCB + q*RSTEPB (16-byte piece tid%KCB)
    const int srow = tid / KC4, sc4 = tid % KC4;
    const int srowb = tid / KCB, scb = tid % KCB;
    int voA[ALD], voA2[ALD], voB[BLD];  // byte offsets of the staged rows (range-checked)
    int ldsB[BLD];                      // MODE 2: LDS dword offset of B piece q within a buffer
    int ldsA[AX6 ? ALD : 1];            // (AX6) LDS dword offset of A piece q, as ldsB
#pragma unroll
    for (int q = 0; q < ALD; ++q) {
        if constexpr (AX6) {  // piece idx: row w / 6, term (w % 6) / 2, k half w % 2 of the tile's contiguous chunk
            const int w = tid + q * NT;
            voA[q] = w < BM * 6 ? w * 16 : 0;
            voA2[q] = 0;
            ldsA[q] = (w / 6) * LS + ((w % 6) >> 1) * (BK / 2) + 4 * (w & 1);
        } else {
            voA[q] = ((srow + q * RSTEP) * p.lda + sc4 * EPA) * ESA;
            voA2[q] = ((srow + q * RSTEP) * p.lda2 + sc4 * EPA) * ESA;
        }
    }
#pragma unroll
    for (int q = 0; q < BLD; ++q) {
        if constexpr (MODE == 2) {
            // a stage is BK/16 image chunks; a chunk's B tile is contiguous ([BN rows][6 pieces of
            // 16 bytes]), consecutive chunks ldb * 96 bytes apart.  Piece idx: chunk h, row w / 6,
            // term (w % 6) / 2, k half w % 2 -> LDS dword term * BK/2 + 8 h + 4 (w % 2) of the row.
            const int idx = tid + q * NT;
            const int h = idx / (BN * 6), w = idx % (BN * 6);
            voB[q] = idx < BN * KCB ? h * p.ldb * 96 + w * 16 : 0;
            ldsB[q] = (w / 6) * LS + ((w % 6) >> 1) * (BK / 2) + 8 * h + 4 * (w & 1);
        } else {
            voB[q] = (srowb + q * RSTEPB) * p.ldb * ESZB + scb * 16;
        }
    }
    // LDS write offsets in dwords: A as fp32 float4 (4 dwords), bf16x4 (2 dwords) or a bf16x8 piece
    // (4 dwords); B 16-byte pieces
    const int lds_a = srow * LS + sc4 * (ABF || !BF ? 4 : 2);
    const int lds_b = srowb * LS + scb * 4;

    floatx4 ra[DEPTH][ALD], rb[DEPTH][BLD];
    // Straight-line staging: every call issues exactly ALD + BLD loads (an empty
    // view when `valid` is false, reads return zero) with no data-dependent branch,
    // so the compiler tracks vmcnt precisely and the LDS writes of one register
    // set wait only for that set's loads, not for the prefetch issued after them.
    auto gload = [&](int set, int kc, int m0, int n0, bool valid) {
        const int k0 = kc * BK;
        const int rows = valid ? min(BM, p.M - m0) : 0;
        const bool second = k0 >= p.K1;  // wave-uniform: A2 half of a virtual concat
        const char* abase = second ? reinterpret_cast<const char*>(p.A2) + (int64_t)m0 * p.lda2 * ESA
                                   : reinterpret_cast<const char*>(cA) + (int64_t)m0 * p.lda * ESA;
        const int ald = second ? p.lda2 : p.lda;
        const int ak = second ? k0 - p.K1 : k0;
        if constexpr (AX6) {  // chunk kc, rows m0 .. m0 + rows - 1: 96 * rows contiguous bytes
            const rsrc_t rA = make_view(reinterpret_cast<const float*>(reinterpret_cast<const char*>(cA) +
                                                                       ((int64_t)kc * p.lda + m0) * 96), rows * 96);
#pragma unroll
            for (int q = 0; q < ALD; ++q) ra[set][q] = bload4(rA, voA[q], 0);
        } else {
        const rsrc_t rA = make_view(reinterpret_cast<const float*>(abase), rows * ald * ESA);
#pragma unroll
        for (int q = 0; q < ALD; ++q) ra[set][q] = bload4(rA, second ? voA2[q] : voA[q], ak * ESA);
        }
        // MODE 2: chunk kc of the image is [ldb rows][48 bf16]; the tile's BN rows are 96 * BN contiguous bytes
        const int64_t bofs = MODE == 2 ? ((int64_t)kc * (BK / 16) * p.ldb + n0) * 96 : (int64_t)n0 * p.ldb * ESZB;
        const rsrc_t rB = make_view(reinterpret_cast<const float*>(reinterpret_cast<const char*>(cB) + bofs),
                                    valid ? (MODE == 2 ? ((BK / 16 - 1) * p.ldb + BN) * 96 : BN * p.ldb * ESZB) : 0);
#pragma unroll
        for (int q = 0; q < BLD; ++q) rb[set][q] = bload4(rB, voB[q], MODE == 2 ? 0 : k0 * ESZB);
    };
    // piece < 0: the whole stage; piece q < ALD: A row q only; piece ALD: B only
    auto lstore = [&](int set, int buf, int piece = -1) {
        float* a = sA + buf * BM * LS + lds_a;
        float* b = sB + buf * BN * LS + lds_b;
#pragma unroll
        for (int q = 0; q < ALD; ++q) {
            if (piece >= 0 && piece != q) continue;
            if constexpr (AX6) {
                if (BM * 6 % NT == 0 || tid + q * NT < BM * 6)  // wave-uniform
                    *reinterpret_cast<floatx4*>(sA + buf * BM * LS + ldsA[q]) = ra[set][q];
            } else if constexpr (MODE == 2) {
                bf16x4 x0, x1, x2;
                split3(ra[set][q], x0, x1, x2);
                *reinterpret_cast<bf16x4*>(a + q * RSTEP * LS) = x0;
                *reinterpret_cast<bf16x4*>(a + q * RSTEP * LS + BK / 2) = x1;
                *reinterpret_cast<bf16x4*>(a + q * RSTEP * LS + BK) = x2;
            } else if constexpr (ABF)
                *reinterpret_cast<floatx4*>(a + q * RSTEP * LS) = ra[set][q];  // 8 bf16 as they are
            else if constexpr (BF)
                *reinterpret_cast<bf16x4*>(a + q * RSTEP * LS) = __builtin_convertvector(ra[set][q], bf16x4);
            else
                *reinterpret_cast<floatx4*>(a + q * RSTEP * LS) = ra[set][q];
        }
#pragma unroll
        for (int q = 0; q < BLD; ++q) {
            if (piece >= 0 && piece != ALD) continue;
            if constexpr (MODE == 2) {
                const int idx = tid + q * NT;
                if (BN * KCB % NT == 0 || idx < BN * KCB)  // wave-uniform (NT, BN*KCB multiples of 64)
                    *reinterpret_cast<floatx4*>(sB + buf * BN * LS + ldsB[q]) = rb[set][q];
            } else {
                *reinterpret_cast<floatx4*>(b + q * RSTEPB * LS) = rb[set][q];
            }
        }
    };
    // flags bit 0: walk the M-tiles last to first (consecutive layers of a chain alternate, so
    // a layer reads first the rows its producer wrote last, still in the memory-side cache)
    const int ntm8 = ((p.n_tiles_m + 7) / 8) * 8;
    auto coords = [&](int vt, int& tm, int& tn) {
        tile_coords(vt, T, tm, tn);
        if (p.flags & 1) tm = ntm8 - 1 - tm;
    };
    auto next_valid = [&](int vt) {
        for (; vt < ntiles; vt += gridDim.x) {
            int tm, tn;
            coords(vt, tm, tn);
            if (tm * BM < p.M) return vt;
        }
        return ntiles;
    };

    // pinned compute/staging segments: the 256x256 bf16x6 tile (one workgroup per CU, so no
    // partner workgroup's MFMAs cover a trailing staging block)
    constexpr bool kSeg = MODE == 2 && TM * TN >= 8 && TN > ALD && DEPTH == 2 && OCC == 1 && BK == 16;
    const int arow = wm * TM * 32 + (lane & 31);
    const int brow = wn * TN * 32 + (lane & 31);
    const int kofs = (BK / 2) * (lane >> 5);
    const int Nmain = (EPI == CN_EPI_MUL && p.nsplit < cN) ? p.nsplit : cN;
    constexpr int C4 = BN / 4;
    constexpr int RPP = NT / C4;
    constexpr int GMAX = OCC >= 3 ? 2 : 4;  // rows of aux loads in flight per thread (VGPR budget)
    constexpr int GROUP = (PROWS / RPP) < GMAX ? (PROWS / RPP) : GMAX;
    static_assert((PROWS / RPP) % GROUP == 0, "epilogue passes");
    constexpr bool kAux0 = EPI == CN_EPI_MUL || EPI == CN_EPI_TANGENT || EPI == CN_EPI_BWD_SOFTPLUS ||
                           EPI == CN_EPI_BWD_RELU;
    constexpr bool kAux1 = EPI == CN_EPI_BWD_SOFTPLUS;  // aux1 = s, aux2 = u' (second-order term)

    // epilogue thread geometry: row rr + k*RPP of the slab, columns 4*c4 .. 4*c4+3
    const int c4 = tid % C4;
    const int rr = tid / C4;
    const int voO0 = (rr * p.ld_out0 + 4 * c4) * 4;
    const int voO1 = (rr * p.ld_out1 + 4 * c4) * 4;
    const int voX0 = (rr * p.ld_aux0 + 4 * c4) * 4;
    const int voX1 = (rr * p.ld_aux1 + 4 * c4) * (AUX12B ? 2 : 4);
    const int voX2 = (rr * p.ld_aux2 + 4 * c4) * (AUX12B ? 2 : 4);
    const int voS = (rr * p.ld_split + 4 * c4) * 4;
    const int voX0b = (rr * p.ld_aux0 + 4 * c4) * 2;  // (AUX0B) bf16 aux0
    const int voO0b = (rr * p.ld_out0_b + 4 * c4) * 2;  // bf16 images of out0 / out1
    const int voO1b = (rr * p.ld_out1_b + 4 * c4) * 2;
    const float c_exp = p.beta * 1.44269504088896341f;        // beta log2(e)
    const float c_thr = p.threshold * 1.44269504088896341f;   // threshold in the log2 domain
    const float c_log = 0.693147180559945309f / p.beta;       // ln(2) / beta

    int vt = next_valid(blockIdx.x);
    if (vt >= ntiles) return;
    if constexpr (TBL > 0) {  // visible after the first tile's staging barrier
        const rsrc_t rbias = make_view(p.bias, kBias && p.bias ? cN * 4 : 0);
        const rsrc_t rcolv = make_view(p.colv, kColv && p.colv ? cN * 4 : 0);
        const rsrc_t rhw = make_view(p.head_w, kHead ? cN * 4 : 0);
        for (int i = tid; i < TBLC / 4; i += NT) {
            if (kBias) *reinterpret_cast<floatx4*>(sBias + 4 * i) = bload4(rbias, 16 * i, 0);
            if (kColv) *reinterpret_cast<floatx4*>(sColv + 4 * i) = bload4(rcolv, 16 * i, 0);
            if (kHead) *reinterpret_cast<floatx4*>(sHeadW + 4 * i) = bload4(rhw, 16 * i, 0);
        }
        if (kHead && tid == 0) sHeadW[TBLC] = p.head_b[0];
    }
    int tm, tn;
    coords(vt, tm, tn);

    // ---- LDS-DMA ring (kDma): wave w < 4 fills A rows 64 w .. + 63, wave w >= 4 B rows 64 (w - 4) ..,
    // four 1-KiB pieces of 16 rows each; lane l: row + (l >> 2), physical chunk l & 3
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)smem);
    const int dwave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool dsb = dwave >= 4;
    const int drow = (dwave & 3) * 64 + (lane >> 2);
    const int dch = (lane & 3) ^ ((lane >> 4) & 3);  // logical chunk of the lane's physical one
    auto ufirst = [](const void* ptr) {
        const uint64_t x = reinterpret_cast<uint64_t>(ptr);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
        return reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    };
    // chunk kc of the tile at (m0, n0) into ring slot `slot` (valid false: zeros)
    auto dma_issue = [&](int slot, int kc, int m0, int n0, bool valid) {
        const int k0 = kc * BK;
        const char* base;
        int ld, bytes, kk;
        if (!dsb) {
            const bool second = k0 >= p.K1;  // wave-uniform: A2 half of a virtual concat
            ld = second ? p.lda2 : p.lda;
            kk = second ? k0 - p.K1 : k0;
            base = reinterpret_cast<const char*>(second ? p.A2 : cA) + (int64_t)m0 * ld * 2;
            bytes = valid ? min(BM, p.M - m0) * ld * 2 : 0;
        } else {
            ld = p.ldb;
            kk = k0;
            base = reinterpret_cast<const char*>(cB) + (int64_t)n0 * ld * 2;
            bytes = valid ? BN * ld * 2 : 0;
        }
        const rsrc_t v = __builtin_amdgcn_make_buffer_rsrc(ufirst(base), 0, __builtin_amdgcn_readfirstlane(bytes),
                                                           0x00020000);
        char* dst = reinterpret_cast<char*>(smem) + slot * DSTAGE + (dsb ? DSIDEA : 0) + (dwave & 3) * 64 * DROWB;
        // (A, read once per tile, non-temporally with CN_DMA_A_NT; the weights stay cached: every workgroup reads them)
        if (CN_DMA_A_NT && !dsb) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(v, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16,
                                                         (drow + 16 * j) * ld * 2 + (kk + dch * 8) * 2, 0, 0, 2);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(v, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16,
                                                         (drow + 16 * j) * ld * 2 + (kk + dch * 8) * 2, 0, 0, 0);
        }
    };
    // MFMA operand reads: lane l's row (l & 31) of each 32-row block, 16-byte chunk 2 ks + (l >> 5)
    // at its swizzled place ((row >> 2) & 3 = ((l & 31) >> 2) & 3: the blocks start at multiples of 32)
    const int dsw = ((lane & 31) >> 2) & 3;
    uint32_t daoff[2], dboff[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int ch = ((2 * ks + (lane >> 5)) ^ dsw) << 4;
        daoff[ks] = lds0 + (wm * TM * 32 + (lane & 31)) * DROWB + ch;
        dboff[ks] = lds0 + DSIDEA + (wn * TN * 32 + (lane & 31)) * DROWB + ch;
    }
    if constexpr (kDma) {
        // the column tables are read into registers now (a table read beside the ring would wait
        // for every DMA in flight); 128 < N <= 256: one N-tile, n0 = 0 on every tile
        __syncthreads();
#pragma unroll
        for (int d = 0; d < DNS - 1; ++d) dma_issue(d, d, tm * BM, tn * BN, true);
    } else {
        // the first DEPTH chunks of a tile are in the register sets when its loop starts (the next
        // tile's are fetched during the current tile's last DEPTH chunks); see the end of the tile
        // loop for the asm re-definition (the sets enter the loop as asm-defined values on both paths)
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) gload(d, d, tm * BM, tn * BN, true);
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
            for (int q = 0; q < ALD; ++q) asm volatile("" : "+v"(ra[d][q]));
#pragma unroll
            for (int q = 0; q < BLD; ++q) asm volatile("" : "+v"(rb[d][q]));
        }
    }
    // (kDma) per-lane column-table values of the direct epilogues, n0 = 0
    float tbias[TN], tcolv[TN], thw[TN];
    float thb = 0.0f;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int c = min(wn * TN * 32 + (lane & 31) + 32 * j, TBLC - 1);
        tbias[j] = kDma && kBias ? sBias[c] : 0.0f;
        tcolv[j] = kDma && kColv ? sColv[c] : 0.0f;
        thw[j] = kDma && kHead ? sHeadW[c] : 0.0f;
    }
    if (kDma && kHead) thb = sHeadW[TBLC];
    const bool epi_big = !kHead || p.out0 || p.out1 || p.out0_b || p.out1_b;  // (kDma) see the main loop
    // (kDma) the ring's waits: chunk kc's pieces are done once at most the ops issued after them are
    // outstanding -- DNS - 2 later chunks (4 pieces each), and for a tile's first DNS - 1 chunks after
    // the first tile also the previous epilogue's >= kEpiMinVmem (a wait of at most 63: the counter)
    constexpr int kRingWait = 4 * (DNS - 2);
    constexpr int kEpiMinVmem = TM * 8 * TN;
    constexpr int kEpiWait = kRingWait + kEpiMinVmem < 63 ? kRingWait + kEpiMinVmem : 63;
    static_assert(!kDma || (kEpiWait > kRingWait && kRingWait + kEpiMinVmem >= kEpiWait),
                  "the epilogue's memory operations must cover the wait past the ring's chunks");
    int gs = 0;             // (kDma) ring slot of the current tile's chunk 0
    bool gs_first = true;   // (kDma) the workgroup's first tile: no epilogue issued before its chunks

    while (vt < ntiles) {
        const int m0 = tm * BM, n0 = tn * BN;
        const int vt_next = next_valid(vt + gridDim.x);
        int tm_next = 0, tn_next = 0;
        if (vt_next < ntiles) coords(vt_next, tm_next, tn_next);

        if constexpr (!kDma) {
            lstore(0, 0);
            __syncthreads();
        }

        floatx16 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

        // side(j) runs after column block j's MFMAs of the 64x128 wave tiles (kSeg: each
        // block a segment pinned by sched_barrier, so the next stage's split and LDS writes
        // handed to side() interleave with that block's MFMAs instead of trailing all of them)
        auto compute = [&](int cur, auto side) {
            if constexpr (MODE == 2) {
                const float* a_base = sA + cur * BM * LS + arow * LS + 4 * (lane >> 5);
                const float* b_base = sB + cur * BN * LS + brow * LS + 4 * (lane >> 5);
                if constexpr (TM * TN >= 8) {
                    // 64x128 wave tiles: the B fragments of one column block at a time (12 VGPRs
                    // instead of 48 live); a single accumulation chain issues back to back
#pragma unroll
                    for (int ks = 0; ks < BK / 16; ++ks) {
                        bf16x8 af[3][TM];
#pragma unroll
                        for (int t = 0; t < 3; ++t)
#pragma unroll
                            for (int i = 0; i < TM; ++i)
                                af[t][i] = *reinterpret_cast<const bf16x8*>(a_base + i * 32 * LS + t * (BK / 2) + ks * 8);
#pragma unroll
                        for (int j = 0; j < TN; ++j) {
                            bf16x8 bj[3];
#pragma unroll
                            for (int t = 0; t < 3; ++t)
                                bj[t] = *reinterpret_cast<const bf16x8*>(b_base + j * 32 * LS + t * (BK / 2) + ks * 8);
                            constexpr int TA[6] = {0, 1, 0, 2, 1, 0};
                            constexpr int TB[6] = {0, 0, 1, 0, 1, 2};
#pragma unroll
                            for (int u = 0; u < 6; ++u)
#pragma unroll
                                for (int i = 0; i < TM; ++i)
                                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[TA[u]][i], bj[TB[u]], acc[i][j],
                                                                                         0, 0, 0);
                            if (ks == BK / 16 - 1) {
                                side(j);
                                if constexpr (kSeg) __builtin_amdgcn_sched_barrier(0);
                            }
                        }
                    }
                    return;
                }
#pragma unroll
                for (int ks = 0; ks < BK / 16; ++ks) {
                    bf16x8 af[3][TM], bf[3][TN];
#pragma unroll
                    for (int t = 0; t < 3; ++t) {
#pragma unroll
                        for (int i = 0; i < TM; ++i)
                            af[t][i] = *reinterpret_cast<const bf16x8*>(a_base + i * 32 * LS + t * (BK / 2) + ks * 8);
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            bf[t][j] = *reinterpret_cast<const bf16x8*>(b_base + j * 32 * LS + t * (BK / 2) + ks * 8);
                    }
                    // term pairs (ta, tb), ta + tb <= 2, in the order the fragments
                    // arrive (t = 0 first): the first MFMAs wait only for a0, b0
                    constexpr int TA[6] = {0, 1, 0, 2, 1, 0};
                    constexpr int TB[6] = {0, 0, 1, 0, 1, 2};
#pragma unroll
                    for (int u = 0; u < 6; ++u)
#pragma unroll
                        for (int i = 0; i < TM; ++i)
#pragma unroll
                            for (int j = 0; j < TN; ++j)
                                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[TA[u]][i], bf[TB[u]][j], acc[i][j],
                                                                                     0, 0, 0);
                }
                return;
            } else if constexpr (BF) {
                // lane half h holds k = 8h + j of each 16-deep MFMA step (8 bf16 = 4 dwords)
                const float* a_base = sA + cur * BM * LS + arow * LS + 4 * (lane >> 5);
                const float* b_base = sB + cur * BN * LS + brow * LS + 4 * (lane >> 5);
#pragma unroll
                for (int ks = 0; ks < BK / 16; ++ks) {
                    bf16x8 af[TM], bf[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
                        af[i] = *reinterpret_cast<const bf16x8*>(a_base + i * 32 * LS + ks * 8);
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        bf[j] = *reinterpret_cast<const bf16x8*>(b_base + j * 32 * LS + ks * 8);
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
                }
                return;
            }
            const float* a_base = sA + cur * BM * LS + arow * LS + kofs;
            const float* b_base = sB + cur * BN * LS + brow * LS + kofs;
#pragma unroll
            for (int q4 = 0; q4 < BK / 8; ++q4) {
                floatx4 af[TM], bf[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[i] = *reinterpret_cast<const floatx4*>(a_base + i * 32 * LS + q4 * 4);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bf[j] = *reinterpret_cast<const floatx4*>(b_base + j * 32 * LS + q4 * 4);
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e], bf[j][e], acc[i][j], 0, 0, 0);
            }
        };

        const int m_next = tm_next * BM, n_next = tn_next * BN;
        const bool has_next = vt_next < ntiles;
        if constexpr (kDma) {
            // chunk kc is in slot (gs + kc) % DNS; the stage issued at kc (DNS - 1 ahead: this tile's
            // chunk kc + DNS - 1 or the next tile's first ones) goes to the slot chunk kc - 1 used
            for (int kc = 0; kc < nk; ++kc) {
                // this wave's pieces of chunk kc landed.  vmcnt retires in issue order, so the wait
                // counts what was issued after them: DNS - 2 later chunks (4 pieces each), and for
                // the first DNS - 1 chunks of a tile after the first, the previous tile's epilogue
                // too (>= kEpiMinVmem loads / stores per wave -- epi_big: the aux epilogues read 128
                // values, the others store 128 fp32 values or 64 image dwords, SOFTPLUS_HEAD may store
                // neither): kEpiWait (63) then, so the epilogue's stores are not drained first
                if (gs_first || !epi_big || kc >= DNS - 1)
                    wait_vmcnt<kRingWait>();
                else
                    wait_vmcnt<kEpiWait>();
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_barrier();  // every wave's pieces landed; chunk kc - 1 consumed
                asm volatile("" ::: "memory");
                const int cn = kc + DNS - 1;
                const bool here = cn < nk;
                dma_issue((gs + cn) % DNS, here ? cn : cn - nk, here ? m0 : m_next, here ? n0 : n_next, here || has_next);
                const uint32_t sb = ((gs + kc) % DNS) * DSTAGE;
                bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
                    for (int i = 0; i < TM; ++i) af[ks][i] = __builtin_bit_cast(bf16x8, lds_read_b128<0>(daoff[ks] + sb + i * 32 * DROWB));
#pragma unroll
                    for (int j = 0; j < TN; ++j) bfr[ks][j] = __builtin_bit_cast(bf16x8, lds_read_b128<0>(dboff[ks] + sb + j * 32 * DROWB));
                }
                static_assert(TM == 2 && TN == 4, "the lgkmcnt split below counts 6 reads per k-step");
                asm volatile("s_waitcnt lgkmcnt(6)"
                             : "+v"(af[0][0]), "+v"(af[0][1]), "+v"(bfr[0][0]), "+v"(bfr[0][1]), "+v"(bfr[0][2]), "+v"(bfr[0][3]));
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bfr[0][j], acc[i][j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(af[1][0]), "+v"(af[1][1]), "+v"(bfr[1][0]), "+v"(bfr[1][1]), "+v"(bfr[1][2]), "+v"(bfr[1][3]));
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
            }
            gs = (gs + nk) % DNS;
            gs_first = false;
        } else if constexpr (DEPTH == 1) {
            for (int kc = 0; kc < nk; ++kc) {
                const int cur = kc & 1;
                // chunk kc+1 of this tile, or the next tile's first chunk (consumed after the epilogue)
                const bool more = kc + 1 < nk;
                gload(0, more ? kc + 1 : 0, more ? m0 : m_next, more ? n0 : n_next, more || has_next);
                compute(cur, [](int) {});
                if (more) lstore(0, cur ^ 1);
                __syncthreads();
            }
        } else {
            // DEPTH register sets: chunks c+1 .. c+DEPTH-1 are in flight while chunk c
            // is computed from LDS buffer c&1; set c%DEPTH (already in LDS) then takes
            // chunk c+DEPTH, or the next tile's chunk c+DEPTH-nk past the end.
            static_assert(DEPTH % 2 == 0, "LDS buffer of chunk kc+j is j&1");
            for (int kc = 0; kc < nk; kc += DEPTH) {
#pragma unroll
                for (int j = 0; j < DEPTH; ++j) {
                    const int cn = kc + j + DEPTH;
                    const bool here = cn < nk;
                    // past this tile: chunk cn - nk of the next one, issued before this tile's
                    // epilogue stores, so the next tile's first DEPTH stagings never wait for them
                    gload(j, here ? cn : cn - nk, here ? m0 : m_next, here ? n0 : n_next, here || has_next);
                    if constexpr (kSeg) {
                        // the next stage's staging (unconditional: after a tile's last chunk it
                        // stages the next tile's first chunk, or zeros, into the free buffer,
                        // which the epilogue parks over and the next tile stages again), one
                        // piece per column block
                        compute(j & 1, [&](int jj) {
                            if (jj <= ALD) lstore((j + 1) % DEPTH, (j + 1) & 1, jj);
                        });
                        __syncthreads();
                        continue;
                    }
                    compute(j & 1, [](int) {});
                    // unconditional (branch-free: compute and the next stage's staging share a
                    // basic block, so the scheduler can interleave the split VALU / LDS writes
                    // with the MFMAs).  After the last chunk this stages the next tile's first
                    // chunk (or zeros) into the free buffer: harmless, the epilogue parks over it
                    // and the next tile stages it again.
                    if (kc + j + 1 < nk) lstore((j + 1) % DEPTH, (j + 1) & 1);
                    __syncthreads();
                }
            }
        }

        // Every staging load is complete by here (the epilogue's registers reuse the idle
        // set's, so the compiler drains them first).  Re-defining the register sets through
        // an empty asm tells it so: the next tile's staging of its prefetched first chunk then
        // waits for nothing, instead of for the epilogue's stores (one vmcnt, in issue order).
        if constexpr (!kDma) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
                for (int q = 0; q < ALD; ++q) asm volatile("" : "+v"(ra[d][q]));
#pragma unroll
                for (int q = 0; q < BLD; ++q) asm volatile("" : "+v"(rb[d][q]));
            }
        }
        // Epilogue: park the accumulator tile (or a slab of PROWS rows of it) in the
        // now free staging LDS, then process it row-wise with 16-byte coalesced
        // buffer loads / stores; every aux load of a group of passes is issued
        // before its math.  C/D layout of the 32x32 MFMA: col = lane&31,
        // row = (r&3) + 8*(r>>2) + 4*(lane>>5).
        const int rows = min(BM, p.M - m0);
        // per-tile views, re-based on the pass's first row by SALU arithmetic (view_at)
        const TileView tO0 = {cOut0 + (int64_t)m0 * p.ld_out0 + n0, p.ld_out0, cOut0 ? (rows * p.ld_out0 - n0) * 4 : 0};
        const TileView tO1 = {p.out1 + (int64_t)m0 * p.ld_out1 + n0, p.ld_out1, p.out1 ? (rows * p.ld_out1 - n0) * 4 : 0};
        const TileView tX0 = AUX0B ? tile_view_b16(p.aux0, p.ld_aux0, m0, n0, rows)
                                  : TileView{p.aux0 + (int64_t)m0 * p.ld_aux0 + n0, p.ld_aux0,
                                             p.aux0 ? (rows * p.ld_aux0 - n0) * 4 : 0};
        // bf16 images of out0 / out1 (MODE 1; empty views when absent)
        const TileView tO0b = tile_view_b16(p.out0_b, p.ld_out0_b, m0, n0, rows);
        const TileView tO1b = tile_view_b16(p.out1_b, p.ld_out1_b, m0, n0, rows);
        const bool has_b0 = MODE == 1 && p.out0_b != nullptr;  // wave-uniform
        const bool has_b1 = MODE == 1 && p.out1_b != nullptr;
        // the direct epilogues skip the fp32 stores of an absent out0 / out1 (a wave-uniform branch:
        // image-only outputs would otherwise issue two dropped stores per stored image dword)
        const bool has_o0 = cOut0 != nullptr, has_o1 = p.out1 != nullptr;
        const TileView tX1 = AUX12B ? tile_view_b16(p.aux1, p.ld_aux1, m0, n0, rows)
                                    : TileView{p.aux1 + (int64_t)m0 * p.ld_aux1 + n0, p.ld_aux1,
                                               p.aux1 ? (rows * p.ld_aux1 - n0) * 4 : 0};
        const TileView tX2 = AUX12B ? tile_view_b16(p.aux2, p.ld_aux2, m0, n0, rows)
                                    : TileView{p.aux2 + (int64_t)m0 * p.ld_aux2 + n0, p.ld_aux2,
                                               p.aux2 ? (rows * p.ld_aux2 - n0) * 4 : 0};
        const TileView tR = {p.rowv + m0, 1, ROWV ? rows * 4 : 0};
        const int sh = n0 - p.nsplit;  // out_split column of this tile's first column
        const TileView tS = {p.out_split + (int64_t)m0 * p.ld_split + sh, p.ld_split,
                             p.out_split ? (rows * p.ld_split - sh) * 4 : 0};

        const bool tile_main = n0 + BN <= Nmain;
        const int col = n0 + 4 * c4;
        const int region = col < Nmain ? 0 : (col < cN ? 1 : (col < cNzero ? 2 : 3));
        // (columns >= N read zeros from the table: their lanes are not region 0 anyway)
        const int tcol = min(col, TBLC - 4);
        floatx4 bias = {0.f, 0.f, 0.f, 0.f}, colv = {0.f, 0.f, 0.f, 0.f}, hw = {0.f, 0.f, 0.f, 0.f};
        if (kBias) bias = *reinterpret_cast<const floatx4*>(sBias + tcol);
        if (kColv) colv = *reinterpret_cast<const floatx4*>(sColv + tcol);
        if (kHead) hw = *reinterpret_cast<const floatx4*>(sHeadW + tcol);
        const float hb = kHead ? sHeadW[TBLC] : 0.0f;
        const TileView tI = {reinterpret_cast<const float*>(p.head_idx) + m0, 1, kHead && p.head_idx ? rows * 4 : 0};
        float* sC = smem;
        // aux rows of an epilogue group, double-buffered: group g+1's loads are issued
        // before group g's stores, so waiting for them never waits for those stores
        // (gfx9's one vmcnt counts loads and stores in issue order); group 0's are
        // issued before the accumulators are parked
        constexpr int NG = PROWS / RPP / GROUP;
        floatx4 x0[2][GROUP], x1[2][GROUP], x2[2][GROUP];
        float rv[2][GROUP];
        int hidx[2][GROUP];
        auto aux_load = [&](int part, int g, int slot) {
#pragma unroll
            for (int q = 0; q < GROUP; ++q) {
                const int lrow = part * PROWS + (g * GROUP + q) * RPP;  // wave-uniform slab row of the pass
                // unconditional: the views make reads past a row (columns >= N) or
                // past the last row harmless, and only region-0 lanes use the values
                if (kAux0) x0[slot][q] = AUX0B ? bload_b16x4(view_at(tX0, lrow), voX0b, 0) : eload4(view_at(tX0, lrow), voX0, 0);
                if (kAux1) x1[slot][q] = AUX12B ? bload_b16x4(view_at(tX1, lrow), voX1, 0) : eload4(view_at(tX1, lrow), voX1, 0);
                if (kAux1) x2[slot][q] = AUX12B ? bload_b16x4(view_at(tX2, lrow), voX2, 0) : eload4(view_at(tX2, lrow), voX2, 0);
                if (ROWV) rv[slot][q] = bload1(view_at(tR, lrow), rr * 4, 0);
                if (kHead) hidx[slot][q] = __builtin_bit_cast(int, bload1(view_at(tI, lrow), rr * 4, 0));
            }
        };
        constexpr bool kAnyAux = kAux0 || kAux1 || ROWV || kHead;
        // main-region values of pass q of a group (the EPI's math on 4 columns)
        auto main_vals = [&](const floatx4& v, int slot, int q, floatx4& o0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                // scaling by 1/adiv, 1/odiv is a multiply by exactly 1.0 when absent:
                // no per-element select for a uniform flag
                float u = v[e] * p.inv_adiv;
                if (ROWV) u = u + rv[slot][q] * colv[e];
                if constexpr (EPI == CN_EPI_STORE) {
                    o0[e] = u + bias[e];
                } else if constexpr (EPI == CN_EPI_SOFTPLUS || kHead) {
                    o0[e] = softplus_hw(u + bias[e], c_exp, c_thr, c_log) * cInvOdiv;
                } else if constexpr (EPI == CN_EPI_RELU) {
                    const float z = u + bias[e];
                    o0[e] = z > 0.0f ? z : 0.0f;
                } else if constexpr (EPI == CN_EPI_MUL) {
                    o0[e] = u * sigma_from_act(x0[slot][q][e], p.aux_c);
                } else if constexpr (EPI == CN_EPI_TANGENT) {
                    o0[e] = u * sigma_from_act(x0[slot][q][e], p.aux_c) * cInvOdiv;
                } else if constexpr (EPI == CN_EPI_BWD_SOFTPLUS) {
                    // Z = v sigma + beta s (1 - sigma) z', with z' = u' / sigma from the
                    // stored tangent u' = sigma z' (aux2_scale = beta * its divisor):
                    // the second-order term of softplus is rebuilt here instead of
                    // being written by the tangent pass and read back.  sigma = 0
                    // implies s = u' = 0 (both carry the factor sigma): term 0.
                    // aux1 / aux2 absent: zero-record views read 0.
                    const float sg = sigma_from_act(x0[slot][q][e], p.aux_c);
                    const float rr = sg > 0.0f ? (1.0f - sg) * __builtin_amdgcn_rcpf(sg) : 0.0f;
                    o0[e] = u * sg + x1[slot][q][e] * x2[slot][q][e] * (p.aux2_scale * rr);
                } else if constexpr (EPI == CN_EPI_BWD_RELU) {
                    o0[e] = x0[slot][q][e] > 0.0f ? u : 0.0f;
                }
            }
        };
        // Two specialisations of the slab passes: MAIN (wave-uniform: every column of the
        // tile is in the main region) stores every pass unconditionally, so each wait for
        // a group's aux rows counts exactly the stores issued after them; the general one
        // (edge tiles: split / zero-fill / untouched columns) branches per lane and ends
        // with the aux registers consumed, so no path carries a pending load into the next
        // tile (where the compiler would drain the vmcnt, epilogue stores included).
        auto consume_aux = [&]() {
#pragma unroll
            for (int sl = 0; sl < 2; ++sl)
#pragma unroll
                for (int q = 0; q < GROUP; ++q) {
                    if (kAux0) asm volatile("" ::"v"(x0[sl][q]));
                    if (kAux1) asm volatile("" ::"v"(x1[sl][q]));
                    if (kAux1) asm volatile("" ::"v"(x2[sl][q]));
                    if (ROWV) asm volatile("" ::"v"(rv[sl][q]));
                    if (kHead) asm volatile("" ::"v"(hidx[sl][q]));
                }
        };
        auto passes = [&](auto main_tag) {
            constexpr bool MAIN = decltype(main_tag)::value;
            if (kAnyAux) aux_load(0, 0, 0);
#pragma unroll
            for (int part = 0; part < NPART; ++part) {
                if (part > 0) __syncthreads();  // previous slab consumed
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int row = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                            if (NPART == 1 || row / PROWS == part)
                                sC[(row - part * PROWS) * CS + wn * TN * 32 + j * 32 + (lane & 31)] = acc[i][j][r];
                        }
                __syncthreads();
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    const int slot = (part * NG + g) & 1;
                    const int pb = g * GROUP;
                    if (kAnyAux) {  // prefetch the next group (or the next part's first)
                        if (g + 1 < NG) aux_load(part, g + 1, slot ^ 1);
                        else if (part + 1 < NPART) aux_load(part + 1, 0, slot ^ 1);
                    }
#pragma unroll
                    for (int q = 0; q < GROUP; ++q) {
                        const int lrow = part * PROWS + (pb + q) * RPP;
                        const floatx4 v = *reinterpret_cast<const floatx4*>(sC + (rr + (pb + q) * RPP) * CS + 4 * c4);
                        floatx4 o0;
                        // the bf16 images of the values stored to out0 / out1 (MODE 1)
                        auto sb0 = [&](const floatx4& w) {
                            if (has_b0) bstore_b16x4(view_at(tO0b, lrow), voO0b, 0, w);
                        };
                        auto sb1 = [&](const floatx4& w) {
                            if (has_b1) bstore_b16x4(view_at(tO1b, lrow), voO1b, 0, w);
                        };
                        const floatx4 zero4 = {0.f, 0.f, 0.f, 0.f};
                        if constexpr (kHead) {  // the row's activation, the ∇-pass seed, the head row-dot
                            float part = 0.0f;
                            if (MAIN || region == 0) {
                                main_vals(v, slot, q, o0);
                                estore4(view_at(tO0, lrow), voO0, 0, o0);  // (out0 NULL: empty view)
                                sb0(o0);
                                floatx4 s1;
#pragma unroll
                                for (int e = 0; e < 4; ++e) {
                                    part += o0[e] * hw[e];
                                    s1[e] = colv[e] * sigma_from_act(o0[e], p.aux_c);
                                }
                                estore4(view_at(tO1, lrow), voO1, 0, s1);  // (out1 NULL: empty view)
                                sb1(s1);
                            } else if (region == 2) {
                                estore4(view_at(tO0, lrow), voO0, 0, zero4);
                                estore4(view_at(tO1, lrow), voO1, 0, zero4);
                                sb0(zero4);
                                sb1(zero4);
                            }
                            // row sum over the C4 lanes holding the row (fixed butterfly order)
#pragma unroll
                            for (int off = C4 / 2; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
                            const int row = m0 + lrow + rr;
                            if (c4 == 0 && row < p.M) {
                                const int dst = p.head_idx ? hidx[slot][q] : row;
                                p.head_out[dst] = part + hb;
                            }
                            continue;
                        }
                        if constexpr (MAIN) {
                            main_vals(v, slot, q, o0);
                            estore4(view_at(tO0, lrow), voO0, 0, o0);
                            sb0(o0);
                        } else if (region == 0) {
                            main_vals(v, slot, q, o0);
                            estore4(view_at(tO0, lrow), voO0, 0, o0);
                            sb0(o0);
                        } else if (region == 1) {  // EPI_MUL split columns: raw (A·Bᵀ)/adiv
#pragma unroll
                            for (int e = 0; e < 4; ++e) o0[e] = v[e] * p.inv_adiv;
                            estore4(view_at(tS, lrow), voS, 0, o0);
                            if (col < cNzero) {
                                estore4(view_at(tO0, lrow), voO0, 0, zero4);
                                sb0(zero4);
                            }
                        } else if (region == 2) {  // zero fill (region 3: past nzero, untouched)
                            estore4(view_at(tO0, lrow), voO0, 0, zero4);
                            sb0(zero4);
                        }
                    }
                }
            }
            if constexpr (!MAIN && kAnyAux) consume_aux();
        };
        // Direct epilogue (main tiles of the aux-free epilogues): every accumulator element
        // goes out from the MFMA layout itself -- lane l holds column l&31 of rows (r&3) +
        // 8(r>>2) + 4(l>>5), so one dword store per (i, j, r) writes two full 128-byte row
        // segments -- with no LDS park, no barrier and no readback.
        // On the 64x128 wave tiles the elementwise aux epilogues (MUL, TANGENT, BWD_SOFTPLUS) go
        // the same way: their aux rows are read in the MFMA layout too (dword loads, two 128-byte
        // row segments per instruction), RG accumulator rows at a time, double-buffered (group
        // g+1's loads issued before group g's stores, so each wait skips those stores)
        constexpr bool kDirectAux = TM * TN >= 8 && !ROWV &&
                                    (EPI == CN_EPI_MUL || EPI == CN_EPI_TANGENT || EPI == CN_EPI_BWD_SOFTPLUS ||
                                     EPI == CN_EPI_BWD_RELU);
        constexpr bool kDirect = !kAnyAux || kDirectAux;
        // SOFTPLUS_HEAD on the 64x128 wave tiles: the activation, the ∇-pass seed and the sdf row-dot
        // from the MFMA layout too (row sums: butterfly over the 32 lanes of a row, then the two
        // column waves' partials through LDS)
        constexpr bool kDirectHead = kHead && TM * TN >= 8;
        // 64x128 wave tiles are dispatched only where one tile spans all columns (128 < N <= 256, no
        // rowv: host-checked), so their kernels carry no LDS-park path (and its registers)
        constexpr bool kDirectOnly = (kDirect || kDirectHead) && TM * TN >= 8;
        // per column block j of this lane: the store offset, or one past any view (the buffer
        // drops the store) for columns >= nzero; live = column < N (else the zero fill of
        // [N, nzero)).  On main tiles every column is live; the 256x256 tile also takes
        // 128 < N < 256 (e.g. the 204-wide layer before the skip, whose row tail holds the
        // embedding: nzero = N there, so those columns are never written)
        auto direct_cols = [&](int vo, int lcol, int* voj, bool* live) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = n0 + lcol + 32 * j;
                voj[j] = col < cNzero ? vo + 128 * j : (1 << 30);
                live[j] = col < cN;
            }
        };
        // bf16 images from the MFMA layout (MODE 1): lanes 2c and 2c + 1 hold columns 2c, 2c + 1 of
        // accumulator rows r (even) and r + 1.  Each lane rounds its own (row r, row r + 1) pair to
        // bf16 (one v_cvt_pk: the RNE of any other packing), the two lanes swap the packed dwords
        // (DPP) and one v_perm picks row r's halves (even lane) or row r + 1's (odd lane): one dword
        // store each, no per-element selects.  Per column block j the lane's byte offset (row r + 1
        // for odd lanes), or one past any view for columns >= nzero (the pair's columns are both
        // below or both past it: nzero % 4 == 0).
        const bool odd = lane & 1;
        // v_perm byte selectors over {recv : own}: own.lo, recv.lo (even); recv.hi, own.hi (odd)
        const unsigned psel = odd ? 0x03020706u : 0x05040100u;
        auto bimg_cols = [&](int ld, int lrow, int lcol, int* vbj) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = lcol - (odd ? 1 : 0) + 32 * j;
                vbj[j] = n0 + c < cNzero ? ((lrow + (odd ? 1 : 0)) * ld + c) * 2 : (1 << 30);
            }
        };
        auto bimg_pair = [&](const TileView& t, int rowi, int vb, float o_r, float o_r1, unsigned sel) {
            const unsigned own = pack_b16x2(o_r, o_r1);
            const unsigned recv = __builtin_amdgcn_mov_dpp(own, 0xB1, 0xF, 0xF, true);  // lane ^ 1
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(recv, own, sel), view_at(t, rowi), vb, 0, CN_EPI_AUX);
        };
        // The direct epilogues take the wave-uniform choices (fp32 out0 stored, bf16 image of it, MUL's
        // split output) as template flags: as branches inside the element loops they left the
        // compiler's vmcnt bookkeeping unsure at every merge point, and it drained vmcnt(0) there --
        // the next tile's staging loads included.
        auto direct_aux = [&](auto o0_tag, auto b0_tag, auto spl_tag) {
            constexpr bool O0 = decltype(o0_tag)::value, B0 = decltype(b0_tag)::value;
            constexpr bool SPL = decltype(spl_tag)::value;
            const int lrow = wm * TM * 32 + 4 * (lane >> 5);
            const int lcol = wn * TN * 32 + (lane & 31);
            const int vo = (lrow * p.ld_out0 + lcol) * 4;
            const int v0 = (lrow * p.ld_aux0 + lcol) * (AUX0B ? 2 : 4);
            const int v1 = (lrow * p.ld_aux1 + lcol) * (AUX12B ? 2 : 4);
            const int v2 = (lrow * p.ld_aux2 + lcol) * (AUX12B ? 2 : 4);
            int voj[TN], vbj[TN];
            bool live[TN];
            direct_cols(vo, lcol, voj, live);
            if (B0) bimg_cols(p.ld_out0_b, lrow, lcol, vbj);
            // EPI_MUL with a split output (the skip layer's ∇ pass: columns [nsplit, N) are the
            // embedding's adjoint, written raw (A·Bᵀ)/adiv to out_split while out0 is zero-filled
            // there; p.nsplit = N without a split)
            bool spl[TN];
            int vsj[TN];
            unsigned keep[TN];  // all ones where out0 takes the epilogue's value (else its zero fill)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = n0 + lcol + 32 * j;
                spl[j] = EPI == CN_EPI_MUL && c >= p.nsplit && c < cN;
                vsj[j] = (lrow * p.ld_split + lcol + 32 * j) * 4;
                keep[j] = live[j] && !spl[j] ? ~0u : 0u;
            }
            // accumulator rows r per group (even: bf16 pairs; one row for the three aux streams of the bf16x6
            // BWD_SOFTPLUS, whose registers the next tile's staging sets share)
            constexpr int RG = kAux1 ? (MODE == 1 ? 2 : 1) : 4;
            constexpr int NGD = TM * 16 / RG;          // groups per tile
            constexpr int ASTEP = AUX0B ? 64 : 128;    // bytes per 32-column block of aux0
            constexpr int XSTEP = AUX12B ? 64 : 128;   // ... of aux1 / aux2
            // raw loaded bits (a bf16 image value is widened where it is used: a widening inside the
            // prefetch would be a use, and the scheduling barrier below would wait for every load)
            unsigned xa[2][RG][TN], xb[2][RG][TN], xc[2][RG][TN];
            auto w0 = [&](unsigned r) { return __builtin_bit_cast(float, AUX0B ? r << 16 : r); };
            auto w12 = [&](unsigned r) { return __builtin_bit_cast(float, AUX12B ? r << 16 : r); };
            auto dload = [&](int g, int sl) {
                const int i = g / (16 / RG), r0 = (g % (16 / RG)) * RG;
#pragma unroll
                for (int q = 0; q < RG; ++q) {
                    const int r = r0 + q, row = i * 32 + (r & 3) + 8 * (r >> 2);
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        xa[sl][q][j] = AUX0B ? eload_u16(view_at(tX0, row), v0, ASTEP * j)
                                            : __builtin_bit_cast(unsigned, eload1(view_at(tX0, row), v0, ASTEP * j));
                        if (kAux1) xb[sl][q][j] = AUX12B ? eload_u16(view_at(tX1, row), v1, XSTEP * j)
                                                         : __builtin_bit_cast(unsigned, eload1(view_at(tX1, row), v1, XSTEP * j));
                        if (kAux1) xc[sl][q][j] = AUX12B ? eload_u16(view_at(tX2, row), v2, XSTEP * j)
                                                         : __builtin_bit_cast(unsigned, eload1(view_at(tX2, row), v2, XSTEP * j));
                    }
                }
            };
            dload(0, 0);
#pragma unroll
            for (int g = 0; g < NGD; ++g) {
                const int sl = g & 1;
                if (g + 1 < NGD) dload(g + 1, sl ^ 1);
                // the next group's loads stay ahead of this group's math (scheduled into it, a load
                // could be followed by its own use and a vmcnt(0): the next tile's staging drained)
                __builtin_amdgcn_sched_barrier(0);
                const int i = g / (16 / RG), r0 = (g % (16 / RG)) * RG;
                float prev[TN];  // row r - 1's stored values (bf16 pairs)
#pragma unroll
                for (int q = 0; q < RG; ++q) {
                    const int r = r0 + q;
                    const int rowi = i * 32 + (r & 3) + 8 * (r >> 2);
                    const rsrc_t vw = view_at(tO0, rowi);
                    float ov[TN];
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const float u = acc[i][j][r] * p.inv_adiv;
                        // the split columns' raw values (a wave-uniform branch; the other lanes' stores
                        // fall past the view), out0 zero-filled there below.  No per-lane branch: the
                        // compiler would sink the aux load into it and drain vmcnt(0) there, the next
                        // tile's staging loads included
                        if constexpr (EPI == CN_EPI_MUL && SPL) estore1(view_at(tS, rowi), spl[j] ? vsj[j] : (1 << 30), 0, u);
                        const float sg = EPI == CN_EPI_BWD_RELU ? 0.0f : sigma_from_act(w0(xa[sl][q][j]), p.aux_c);
                        float o;
                        if constexpr (EPI == CN_EPI_BWD_RELU) {
                            o = w0(xa[sl][q][j]) > 0.0f ? u : 0.0f;
                        } else if constexpr (EPI == CN_EPI_MUL) {
                            o = u * sg;
                        } else if constexpr (EPI == CN_EPI_TANGENT) {
                            o = u * sg * cInvOdiv;
                        } else {  // BWD_SOFTPLUS, as main_vals
                            const float rr2 = sg > 0.0f ? (1.0f - sg) * __builtin_amdgcn_rcpf(sg) : 0.0f;
                            o = u * sg + w12(xb[sl][q][j]) * w12(xc[sl][q][j]) * (p.aux2_scale * rr2);
                        }
                        // (a bit mask, not a select: the compiler made the select a branch per element)
                        ov[j] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, o) & keep[j]);
                        if constexpr (O0) estore1(vw, voj[j], 0, ov[j]);
                    }
                    if constexpr (B0) {
                        if (r & 1) {
#pragma unroll
                            for (int j = 0; j < TN; ++j) bimg_pair(tO0b, rowi - 1, vbj[j], prev[j], ov[j], psel);
                        } else {
#pragma unroll
                            for (int j = 0; j < TN; ++j) prev[j] = ov[j];
                        }
                    }
                }
            }
        };
        auto direct_plain = [&](auto o0_tag, auto b0_tag) {
            constexpr bool O0 = decltype(o0_tag)::value, B0 = decltype(b0_tag)::value;
            const int lrow = wm * TM * 32 + 4 * (lane >> 5);
            const int lcol = wn * TN * 32 + (lane & 31);
            const int vo = (lrow * p.ld_out0 + lcol) * 4;
            int voj[TN], vbj[TN];
            bool live[TN];
            direct_cols(vo, lcol, voj, live);
            if (B0) bimg_cols(p.ld_out0_b, lrow, lcol, vbj);
            // image only (no fp32 out0) on the LDS-DMA tile: columns [N, nzero) zero-filled through the
            // v_perm selector (0x0c: a zero byte) of each half of the lane's dword (columns c, c + 1:
            // c = lcol for even lanes, lcol - 1 for odd ones) instead of a select per element.  (Not on
            // the register-staged tiles: there the compiler answered it with vmcnt(0) waits that drain
            // the next tile's prefetch.)
            constexpr bool kSel = B0 && !O0 && kDma;
            unsigned selj[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = n0 + lcol - (odd ? 1 : 0) + 32 * j;
                selj[j] = (c < cN ? (psel & 0xffffu) : 0x0c0cu) | (c + 1 < cN ? (psel & 0xffff0000u) : 0x0c0c0000u);
            }
            float bj[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) bj[j] = kDma ? tbias[j] : kBias ? sBias[min(n0 + lcol + 32 * j, kTblCols - 1)] : 0.0f;
            float prev[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rowi = i * 32 + (r & 3) + 8 * (r >> 2);
                    const rsrc_t vw = view_at(tO0, rowi);
                    float ov[TN];
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const float z = acc[i][j][r] * p.inv_adiv + bj[j];
                        float o;
                        if constexpr (EPI == CN_EPI_SOFTPLUS) o = softplus_hw(z, c_exp, c_thr, c_log) * cInvOdiv;
                        else if constexpr (EPI == CN_EPI_RELU) o = z > 0.0f ? z : 0.0f;
                        else o = z;
                        ov[j] = kSel ? o : live[j] ? o : 0.0f;
                        if constexpr (O0) estore1(vw, voj[j], 0, ov[j]);
                    }
                    if constexpr (B0) {
                        if (r & 1) {
#pragma unroll
                            for (int j = 0; j < TN; ++j) bimg_pair(tO0b, rowi - 1, vbj[j], prev[j], ov[j], kSel ? selj[j] : psel);
                        } else {
#pragma unroll
                            for (int j = 0; j < TN; ++j) prev[j] = ov[j];
                        }
                    }
                }
        };
        auto direct_head = [&]() {
            const int lrow = wm * TM * 32 + 4 * (lane >> 5);
            const int lcol = wn * TN * 32 + (lane & 31);
            int voj[TN], vo1[TN], vbj[TN], vb1[TN];
            bool live[TN];
            direct_cols((lrow * p.ld_out0 + lcol) * 4, lcol, voj, live);
            if (has_b0) bimg_cols(p.ld_out0_b, lrow, lcol, vbj);
            if (has_b1) bimg_cols(p.ld_out1_b, lrow, lcol, vb1);
            float bj[TN], cj[TN], hj[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = min(n0 + lcol + 32 * j, TBLC - 1);
                bj[j] = kDma ? tbias[j] : sBias[c];
                cj[j] = kDma ? tcolv[j] : sColv[c];
                hj[j] = kDma ? thw[j] : sHeadW[c];  // zero past N (the table's view ends at N)
                vo1[j] = voj[j] == (1 << 30) ? voj[j] : (lrow * p.ld_out1 + lcol + 32 * j) * 4;
            }
            // staging buffer 1 is free after the main loop (its last reader); the DMA ring is not
            float* sRed = kDma ? smem + DNS * DSTAGE / 4 : sA + BM * LS;
            float prev0[TN], prev1[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rowi = i * 32 + (r & 3) + 8 * (r >> 2);
                    const rsrc_t vw = view_at(tO0, rowi);
                    const rsrc_t vw1 = view_at(tO1, rowi);
                    float part = 0.0f;
                    float ov0[TN], ov1[TN];
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const float a = softplus_hw(acc[i][j][r] * p.inv_adiv + bj[j], c_exp, c_thr, c_log) * cInvOdiv;
                        const float o = live[j] ? a : 0.0f;
                        ov0[j] = o;
                        ov1[j] = live[j] ? cj[j] * sigma_from_act(a, p.aux_c) : 0.0f;
                        if (has_o0) estore1(vw, voj[j], 0, o);
                        if (has_o1) estore1(vw1, vo1[j], 0, ov1[j]);
                        part += o * hj[j];
                    }
                    if (has_b0 || has_b1) {
                        if (r & 1) {
#pragma unroll
                            for (int j = 0; j < TN; ++j) {
                                if (has_b0) bimg_pair(tO0b, rowi - 1, vbj[j], prev0[j], ov0[j], psel);
                                if (has_b1) bimg_pair(tO1b, rowi - 1, vb1[j], prev1[j], ov1[j], psel);
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < TN; ++j) {
                                prev0[j] = ov0[j];
                                prev1[j] = ov1[j];
                            }
                        }
                    }
                    // the 32 lanes holding this row (lane >> 5 fixed), fixed butterfly order
#pragma unroll
                    for (int off = 16; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
                    if ((lane & 31) == 0) sRed[(lrow + rowi) * 2 + wn] = part;
                }
            __syncthreads();  // (the next tile's first staging barrier orders these reads before buffer 1's reuse)
            if (tid < BM) {
                const int row = m0 + tid;
                if (row < p.M) {
                    const float sum = sRed[tid * 2] + sRed[tid * 2 + 1];
                    const int dst = p.head_idx ? p.head_idx[row] : row;
                    p.head_out[dst] = sum + (kDma ? thb : sHeadW[TBLC]);
                }
            }
        };
        using T1 = std::true_type;
        using F0 = std::false_type;
        // out0 or its image out0_b is present (host-checked): no instance without stores, so every
        // epilogue issues at least TM * 8 * TN vector-memory operations per wave (one image dword per
        // row pair and column block), which the LDS-DMA ring's vmcnt(63) relies on (kEpiMinVmem;
        // tools/isa_check.py verifies it on the built ISA)
        auto run_direct_plain = [&]() {
            if (has_o0) {
                if (has_b0) direct_plain(T1{}, T1{}); else direct_plain(T1{}, F0{});
            } else {
                direct_plain(F0{}, T1{});
            }
        };
        auto run_direct_aux = [&]() {
            auto go = [&](auto spl) {
                if (has_o0) {
                    if (has_b0) direct_aux(T1{}, T1{}, spl); else direct_aux(T1{}, F0{}, spl);
                } else {
                    direct_aux(F0{}, T1{}, spl);
                }
            };
            if constexpr (EPI == CN_EPI_MUL) {
                if (p.nsplit < cN) go(T1{}); else go(F0{});
            } else {
                go(F0{});
            }
        };
        if constexpr (kDirectOnly) {
            if constexpr (kDirectHead) direct_head();
            else if constexpr (kDirectAux) run_direct_aux();
            else run_direct_plain();
        } else {
            if (kDirectAux && tile_main) {
                run_direct_aux();
            } else if (kDirect && tile_main) {
                run_direct_plain();
            } else {
                if (tile_main) passes(std::true_type{});
                else passes(std::false_type{});
                __syncthreads();  // sC is the next tile's staging buffer
            }
        }
        vt = vt_next;
        tm = tm_next;
        tn = tn_next;
    }
    // (kDma) the last stages (zeros) land in LDS before the workgroup ends
    if constexpr (kDma) wait_vmcnt<0>();
}



// ---------------------------------------------------------------------------
// Per-row heads: out[dst(m)][c] = act(sum_k A[m][k] W[c][k] + b[c]).  A row is
// read by a 16-lane group (lane g holds columns 4g + 64j, j < 4: four coalesced
// 256-byte segments), so a wavefront covers 4 rows per pass and 2 passes are
// unrolled: 8 independent 16-byte loads per lane in flight.  The 16 partial sums
// of a row meet in a fixed xor-shuffle tree (deterministic).
__global__ void __launch_bounds__(256) row_head_kernel(int M, int K, const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ W, int64_t ldw,
                                                       const float* __restrict__ b, int C, int act, float* out,
                                                       int64_t ld_out, const int* dst) {
    const int lane = threadIdx.x & 63;
    const int g = lane & 15;   // column group of the lane
    const int sub = lane >> 4; // row of the wave's 4-row pass
    const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    floatx4 wv[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 4 * g + 64 * j;
            wv[c][j] = (c < C && k < K) ? *reinterpret_cast<const floatx4*>(W + c * ldw + k) : floatx4{0.f, 0.f, 0.f, 0.f};
        }
    float bias[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) bias[c] = (b && c < C) ? b[c] : 0.0f;
    constexpr int U = 2;  // 4-row passes per iteration
    for (int64_t m0 = wave0 * 4 * U; m0 < M; m0 += nw * 4 * U) {
        floatx4 a[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t m = m0 + 4 * u + sub;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = 4 * g + 64 * j;
                a[u][j] = (m < M && k < K) ? *reinterpret_cast<const floatx4*>(A + m * lda + k) : floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float s[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float t = 0.0f;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    t += (a[u][j][0] * wv[c][j][0] + a[u][j][1] * wv[c][j][1]) + (a[u][j][2] * wv[c][j][2] + a[u][j][3] * wv[c][j][3]);
                s[c] = t;
            }
#pragma unroll
            for (int off = 8; off > 0; off >>= 1)
#pragma unroll
                for (int c = 0; c < 4; ++c) s[c] += __shfl_xor(s[c], off);
            const int64_t m = m0 + 4 * u + sub;
            if (g < C && m < M) {
                float v = s[0];
#pragma unroll
                for (int c = 1; c < 4; ++c)
                    if (g == c) v = s[c];
                v = v + bias[g];
                if (act == 1) v = sigmoidf_ref(v);
                const int64_t o = dst ? (int64_t)dst[m] : m;
                out[o * ld_out + g] = v;
            }
        }
    }
}

// out[m][n] = X[m][n] * w[n], float4-vectorized (N, the leading dimensions and
// the pointers are multiples of 4 floats / 16-byte aligned: checked by the host).
__global__ void __launch_bounds__(256) scale_cols_kernel(int M, int N4, const float* __restrict__ X, int64_t ldx,
                                                         const float* __restrict__ w, const float* __restrict__ rowv,
                                                         float* out, int64_t ldo, float aux_c) {
    const int64_t tot = (int64_t)M * N4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += stride) {
        const int64_t m = idx / N4;
        const int n = (int)(idx - m * N4) * 4;
        floatx4 x = *reinterpret_cast<const floatx4*>(X + m * ldx + n);
        const floatx4 s = *reinterpret_cast<const floatx4*>(w + n);
        if (aux_c != 0.0f)  // X holds softplus outputs: scale softplus' = 1 - exp(-beta X)
            for (int e = 0; e < 4; ++e) x[e] = sigma_from_act(x[e], aux_c);
        floatx4 y = x * s;
        if (rowv) y = y * rowv[m];
        *reinterpret_cast<floatx4*>(out + m * ldo + n) = y;
    }
}

// 4 values at element offset i of an fp32 output, or of its bf16 operand image (ob)
// four consecutive values of a row: fp32, or (B) a bf16 operand image widened
template <bool B>
#ifndef CN_STREAM_NT
#define CN_STREAM_NT 1  // the elementwise adjoint's rows read / written non-temporally (profiles/r6_ab.txt r6w)
#endif
__device__ __forceinline__ floatx4 load_row4(const void* p, int64_t i) {
    if constexpr (B) {
        const u32x2_t* a = reinterpret_cast<const u32x2_t*>(static_cast<const bf16_t*>(p) + i);
        const u32x2_t w = CN_STREAM_NT ? __builtin_nontemporal_load(a) : *a;
        return floatx4{__builtin_bit_cast(float, w[0] << 16), __builtin_bit_cast(float, w[0] & 0xffff0000u),
                       __builtin_bit_cast(float, w[1] << 16), __builtin_bit_cast(float, w[1] & 0xffff0000u)};
    } else {
        const floatx4* a = reinterpret_cast<const floatx4*>(static_cast<const float*>(p) + i);
        return CN_STREAM_NT ? __builtin_nontemporal_load(a) : *a;
    }
}
__device__ __forceinline__ void store_row4(void* out, bool ob, int64_t i, floatx4 v) {
    if (ob) {
        bf16x4* a = reinterpret_cast<bf16x4*>(static_cast<bf16_t*>(out) + i);
        const bf16x4 b = __builtin_convertvector(v, bf16x4);
        if (CN_STREAM_NT)
            __builtin_nontemporal_store(b, a);
        else
            *a = b;
    } else {
        floatx4* a = reinterpret_cast<floatx4*>(static_cast<float*>(out) + i);
        if (CN_STREAM_NT)
            __builtin_nontemporal_store(v, a);
        else
            *a = v;
    }
}

// Adjoint of a softplus layer without a GEMM, when the upstream gradient of its output
// is already at hand (the SDF's last hidden layer once the feature head is folded into
// the colour network):  out = (D + rowv (x) colv) * sg + aux1 * aux2 * c2 * (1 - sg) / sg,
// sg = softplus' recovered from the activation (sigma_from_act); absent terms are 0.
// IB bit 0: D, bit 1: act, bit 2: aux1 / aux2 are bf16 operand images (config C3's bf16 mode)
template <int IB>
__global__ void __launch_bounds__(256) softplus_adjoint_kernel(int M, int N4, const void* __restrict__ D, int64_t ldd,
                                                               const void* __restrict__ act, int64_t lda, float aux_c,
                                                               const float* __restrict__ rowv,
                                                               const float* __restrict__ colv,
                                                               const void* __restrict__ aux1, int64_t ld1,
                                                               const void* __restrict__ aux2, int64_t ld2, float c2,
                                                               void* out, int64_t ldo, bool ob) {
    const int64_t tot = (int64_t)M * N4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += stride) {
        const int64_t m = idx / N4;
        const int n = (int)(idx - m * N4) * 4;
        const floatx4 a = load_row4<(IB & 2) != 0>(act, m * lda + n);
        floatx4 g = D ? load_row4<(IB & 1) != 0>(D, m * ldd + n) : floatx4{0.f, 0.f, 0.f, 0.f};
        if (rowv) g = g + rowv[m] * *reinterpret_cast<const floatx4*>(colv + n);
        floatx4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
        if (aux1) {
            s1 = load_row4<(IB & 4) != 0>(aux1, m * ld1 + n);
            s2 = load_row4<(IB & 4) != 0>(aux2, m * ld2 + n);
        }
        floatx4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float sg = sigma_from_act(a[e], aux_c);
            const float rr = sg > 0.0f ? (1.0f - sg) * __builtin_amdgcn_rcpf(sg) : 0.0f;
            o[e] = g[e] * sg + s1[e] * s2[e] * (c2 * rr);
        }
        store_row4(out, ob, m * ldo + n, o);
    }
}

// The same with the column sums of the sdf row of lin8's weight gradient: a block owns a
// contiguous slab of rows and all N columns (256 threads = 256/(N/4) row lanes x N/4 float4
// columns), accumulates Σ_m rowv[m] act[m][n] + aux2[m][n] per thread in fp32, combines its
// row lanes in a fixed order through LDS and writes one partial row per block.
constexpr int kSaRows = 512;  // rows per block of the column-sum form
template <int IB>
__global__ void __launch_bounds__(256) softplus_adjoint_cs_kernel(int M, int N4, const void* __restrict__ D,
                                                                  int64_t ldd, const void* __restrict__ act,
                                                                  int64_t lda, float aux_c,
                                                                  const float* __restrict__ rowv,
                                                                  const float* __restrict__ colv,
                                                                  const void* __restrict__ aux1, int64_t ld1,
                                                                  const void* __restrict__ aux2, int64_t ld2,
                                                                  float c2, void* out, int64_t ldo, bool ob,
                                                                  float* part, float* rpart) {
    __shared__ floatx4 red[256];
    __shared__ float redr[256];
    const int c = threadIdx.x % N4;
    const int rl = threadIdx.x / N4;
    const int nrl = 256 / N4;
    const int n = 4 * c;
    const int m0 = blockIdx.x * kSaRows, m1 = min(M, m0 + kSaRows);
    const floatx4 cv = colv ? *reinterpret_cast<const floatx4*>(colv + n) : floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 cs = {0.f, 0.f, 0.f, 0.f};
    float rs = 0.0f;  // Σ rowv over the rows of this lane (the head bias gradient), column-0 lanes
    auto row = [&](int m) {
        const floatx4 a = load_row4<(IB & 2) != 0>(act, (int64_t)m * lda + n);
        floatx4 g = D ? load_row4<(IB & 1) != 0>(D, (int64_t)m * ldd + n) : floatx4{0.f, 0.f, 0.f, 0.f};
        const float rv = rowv ? rowv[m] : 0.0f;
        g = g + rv * cv;
        floatx4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
        if (aux1) {
            s1 = load_row4<(IB & 4) != 0>(aux1, (int64_t)m * ld1 + n);
            s2 = load_row4<(IB & 4) != 0>(aux2, (int64_t)m * ld2 + n);
        }
        floatx4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float sg = sigma_from_act(a[e], aux_c);
            const float rr = sg > 0.0f ? (1.0f - sg) * __builtin_amdgcn_rcpf(sg) : 0.0f;
            o[e] = g[e] * sg + s1[e] * s2[e] * (c2 * rr);
        }
        store_row4(out, ob, (int64_t)m * ldo + n, o);
        cs = cs + rv * a + s2;
        rs += rv;
    };
    if (rl < nrl) {
        int m = m0 + rl;
        for (; m + nrl < m1; m += 2 * nrl) {  // two rows in flight per lane (row order of the sums kept)
            row(m);
            row(m + nrl);
        }
        if (m < m1) row(m);
    }
    red[threadIdx.x] = cs;
    redr[threadIdx.x] = rs;
    __syncthreads();
    if (rl == 0) {
        floatx4 t = red[c];
        float tr = redr[c];
        for (int r = 1; r < nrl; ++r) {
            t = t + red[r * N4 + c];
            tr += redr[r * N4 + c];
        }
        *reinterpret_cast<floatx4*>(part + (int64_t)blockIdx.x * N4 * 4 + n) = t;
        if (c == 0 && rpart) rpart[blockIdx.x] = tr;
    }
}

// ---------------------------------------------------------------------------
// Colour head backward: sigmoid + Linear(256 -> 3) (neus_fields.py:367-373).
// Block = 256 threads = 4 row lanes x 64 float4 column groups (K <= 256) over a slice of
// rows; the per-row sigmoid' factors are staged in LDS once, the row lanes' partial dW3 /
// db3 sums meet in a fixed order.
constexpr int kHeadRowsPerBlock = 256;

__global__ void __launch_bounds__(256) rgb_head_bwd_kernel(int M, int K, const float* __restrict__ drgb,
                                                           const float* __restrict__ rgb,
                                                           const float* __restrict__ H3, int64_t ld_h,
                                                           const float* __restrict__ W3, void* dZ2, int64_t ld_dz,
                                                           bool dz_bf16, float* part /*[nblk][4][K]*/) {
    __shared__ float sd[kHeadRowsPerBlock][3];
    __shared__ floatx4 red[4][64][3];
    __shared__ float redb[4][3];
    const int tid = threadIdx.x;
    const int m0 = blockIdx.x * kHeadRowsPerBlock;
    const int m1 = min(M, m0 + kHeadRowsPerBlock);
    for (int i = tid; i < (m1 - m0) * 3; i += 256) {
        const int64_t q = 3 * (int64_t)m0 + i;
        const float y = rgb[q];
        sd[i / 3][i % 3] = drgb[q] * (1.0f - y) * y;  // torch sigmoid_backward: grad * (1 - y) * y
    }
    __syncthreads();
    const int c4 = tid & 63, rl = tid >> 6;
    const int k = 4 * c4;
    const bool kv = k < K;
    floatx4 w0 = {0.f, 0.f, 0.f, 0.f}, w1 = w0, w2 = w0;
    if (kv) {
        w0 = *reinterpret_cast<const floatx4*>(W3 + k);
        w1 = *reinterpret_cast<const floatx4*>(W3 + K + k);
        w2 = *reinterpret_cast<const floatx4*>(W3 + 2 * K + k);
    }
    floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0;
    float b0 = 0.f, b1 = 0.f, b2 = 0.f;
    for (int m = m0 + rl; m < m1; m += 4) {
        const float d0 = sd[m - m0][0], d1 = sd[m - m0][1], d2 = sd[m - m0][2];
        if (kv) {
            const floatx4 h = *reinterpret_cast<const floatx4*>(H3 + (int64_t)m * ld_h + k);
            floatx4 dz;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float dh = d0 * w0[e] + d1 * w1[e] + d2 * w2[e];
                dz[e] = h[e] > 0.0f ? dh : 0.0f;
            }
            if (dz_bf16)  // (bf16 mode: dZ2's image, the operand of the next adjoint GEMM and a weight gradient)
                *reinterpret_cast<bf16x4*>(static_cast<bf16_t*>(dZ2) + (int64_t)m * ld_dz + k) = __builtin_convertvector(dz, bf16x4);
            else
                *reinterpret_cast<floatx4*>(static_cast<float*>(dZ2) + (int64_t)m * ld_dz + k) = dz;
            a0 = a0 + d0 * h;
            a1 = a1 + d1 * h;
            a2 = a2 + d2 * h;
        }
        b0 += d0;
        b1 += d1;
        b2 += d2;
    }
    red[rl][c4][0] = a0;
    red[rl][c4][1] = a1;
    red[rl][c4][2] = a2;
    if (c4 == 0) {
        redb[rl][0] = b0;
        redb[rl][1] = b1;
        redb[rl][2] = b2;
    }
    __syncthreads();
    float* pb = part + (int64_t)blockIdx.x * 4 * K;
    if (rl == 0 && kv) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const floatx4 t = ((red[0][c4][c] + red[1][c4][c]) + red[2][c4][c]) + red[3][c4][c];
            *reinterpret_cast<floatx4*>(pb + c * K + k) = t;
        }
    }
    if (tid < 3) pb[3 * K + tid] = ((redb[0][tid] + redb[1][tid]) + redb[2][tid]) + redb[3][tid];
}


// Column sums over row slices: a workgroup = 64 float4 column groups x 4 row
// groups, LDS combine; slabs then summed by slab_reduce in a fixed order.
constexpr int kColsumRows = 1024;

__global__ void __launch_bounds__(256) colsum_kernel(int M, int K, const float* __restrict__ w,
                                                     const float* __restrict__ X, int64_t ldx, float* part) {
    __shared__ float red[4][256];
    const int c = (blockIdx.y * 64 + (threadIdx.x & 63)) * 4;
    const int rg = threadIdx.x >> 6;
    const int m0 = blockIdx.x * kColsumRows;
    const int m1 = min(M, m0 + kColsumRows);
    // four independent row streams per thread (rows m0 + rg + 4i, by i mod 4), combined in a fixed order
    floatx4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const bool vec = (c + 3 < K) && (ldx % 4 == 0);
    if (c < K) {
        for (int mb = m0 + rg; mb < m1; mb += 16) {
            floatx4 x[4];
            float wm[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = mb + 4 * u;
                const bool in = m < m1;
                if (vec) {
                    x[u] = in ? *reinterpret_cast<const floatx4*>(X + (int64_t)m * ldx + c) : floatx4{0.f, 0.f, 0.f, 0.f};
                } else {
                    for (int e = 0; e < 4; ++e) x[u][e] = (in && c + e < K) ? X[(int64_t)m * ldx + c + e] : 0.0f;
                }
                wm[u] = (w && in) ? w[m] : 1.0f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                for (int e = 0; e < 4; ++e) acc[u][e] += w ? wm[u] * x[u][e] : x[u][e];
        }
    }
    const floatx4 a = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    for (int e = 0; e < 4; ++e) red[rg][(threadIdx.x & 63) * 4 + e] = a[e];
    __syncthreads();
    if (rg == 0 && c < K) {
        for (int e = 0; e < 4 && c + e < K; ++e) {
            const int t = (threadIdx.x & 63) * 4 + e;
            part[(int64_t)blockIdx.x * K + c + e] = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
        }
    }
}


}  // namespace cn

using namespace cn;

// The CU count of the current device (cached per device: the launches size their persistent
// grids from it).
static int device_cus() {
    static thread_local int cached_dev = -1, cached_cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev != cached_dev) {
        int v = 0;
        cached_cus = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
        cached_dev = dev;
    }
    return cached_cus;
}

template <int WM, int WN, int TM, int TN, int BK, int OCC, int DEPTH, int MODE_>
static int launch_linear_tile_m(const cn_linear_desc* d, LinearArgs& a, hipStream_t s) {
    constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN;
    if (d->epilogue == CN_EPI_SOFTPLUS_HEAD && d->N > BN) {
        set_error("cn_linear: SOFTPLUS_HEAD with N=%d needs a tile of >= N columns (this mode / tile: %d)", d->N, BN);
        return CN_ERR_UNSUPPORTED;
    }
    a.n_tiles_m = cdiv(d->M, BM);
    a.n_tiles_n = cdiv(d->N, BN);
    const int ntiles = cdiv(a.n_tiles_m, 8) * 8 * a.n_tiles_n;
    const int grid = std::min(ntiles, OCC * device_cus());  // OCC resident workgroups per CU
    dim3 block(64 * WM * WN);
    // (bf16 aux images -- MODE_ bit 3 -- only for MUL / TANGENT / BWD_SOFTPLUS / BWD_RELU, without a rank-1 term; the
    // 64x128 wave tiles never take a rank-1 term: both host-checked, so those kernels are not built)
    constexpr bool kRowv = (MODE_ & 8) == 0 && TM * TN < 8;
    switch (d->epilogue) {
#define CN_EPI_CASE(E)                                                                                   \
        case E:                                                                                          \
            if constexpr ((MODE_ & 8) == 0 || E == CN_EPI_BWD_RELU || E == CN_EPI_BWD_SOFTPLUS ||       \
                          E == CN_EPI_MUL || E == CN_EPI_TANGENT) {                                      \
                if (kRowv && d->rowv)                                                                    \
                    linear_kernel<WM, WN, TM, TN, BK, OCC, DEPTH, E, kRowv, MODE_><<<grid, block, 0, s>>>(a); \
                else                                                                                     \
                    linear_kernel<WM, WN, TM, TN, BK, OCC, DEPTH, E, false, MODE_><<<grid, block, 0, s>>>(a); \
            }                                                                                            \
            break;
        CN_EPI_CASE(CN_EPI_STORE)
        CN_EPI_CASE(CN_EPI_SOFTPLUS)
        CN_EPI_CASE(CN_EPI_RELU)
        CN_EPI_CASE(CN_EPI_MUL)
        CN_EPI_CASE(CN_EPI_TANGENT)
        CN_EPI_CASE(CN_EPI_BWD_SOFTPLUS)
        CN_EPI_CASE(CN_EPI_BWD_RELU)
        CN_EPI_CASE(CN_EPI_SOFTPLUS_HEAD)
#undef CN_EPI_CASE
        default: set_error("cn_linear: bad epilogue %d", d->epilogue); return CN_ERR_ARG;
    }
    return check_launch("cn_linear");
}

// The template MODE_ of a descriptor on a tile of GEMM mode MODE: + 4 for bf16 A images, + 8 for a
// bf16 aux0 (MODE 1 only).
static int linear_mode_bits(const cn_linear_desc* d, int mode) {
    if (mode == 2) return mode + (d->a_bf16 ? 16 : 0);  // (CN_AB_X6_AIMG) a bf16x6 term image of A
    return mode == 1 ? mode + (d->a_bf16 ? 4 : 0) + (d->aux0_bf16 || d->aux12_bf16 ? 8 : 0) : mode;
}

// measurement build only (-DCN_AB_X6_AIMG=1, profiles/r6_ab.txt): cn_linear reads A as a bf16x6 term image on the
// 256x256 tile (a_bf16 set with CN_MFMA_F32_BF16X6; the layout of split_bf16x3's B images)
#ifndef CN_AB_X6_AIMG
#define CN_AB_X6_AIMG 0
#endif

template <int WM, int WN, int TM, int TN, int BK, int OCC, int DEPTH, int MODE = 0>
static int launch_linear_tile(const cn_linear_desc* d, LinearArgs& a, hipStream_t s) {
    if constexpr (MODE == 2 && CN_AB_X6_AIMG && BK == 16 && TM * TN >= 8) {
        if (linear_mode_bits(d, MODE) == 18) return launch_linear_tile_m<WM, WN, TM, TN, BK, OCC, DEPTH, 18>(d, a, s);
    }
    if constexpr (MODE == 1) {
        switch (linear_mode_bits(d, MODE)) {
            case 5: return launch_linear_tile_m<WM, WN, TM, TN, BK, OCC, DEPTH, 5>(d, a, s);
            case 9: return launch_linear_tile_m<WM, WN, TM, TN, BK, OCC, DEPTH, 9>(d, a, s);
            case 13: return launch_linear_tile_m<WM, WN, TM, TN, BK, OCC, DEPTH, 13>(d, a, s);
            default: break;
        }
    }
    return launch_linear_tile_m<WM, WN, TM, TN, BK, OCC, DEPTH, MODE>(d, a, s);
}


// The kernel instance cn_linear launches for a descriptor: ONE function decides it, for the
// launch and for cn_linear_kernel_name (a profiler's name of the launch), so the two cannot
// disagree.  X-macro rows: (tile, WM, WN, TM, TN, BK, OCC, DEPTH, MODE).
//   bf16x6 tiles (measured at C2's layer shape, M = 524,288, N = K = 256):
//   * SQ 256x256, 8 waves of 64x128, 1 / CU, 16-deep stages: whole 256-wide rows per workgroup (A
//     read and split once), direct epilogues (STORE / SOFTPLUS / RELU / MUL incl. the split output /
//     TANGENT / BWD_RELU / SOFTPLUS_HEAD) for 128 < N <= 256, K >= 128.  Main loop 316-320 us vs 374
//     on 256x128; SOFTPLUS 445 vs 480-509, RELU 385 vs 408-420, MUL / TANGENT 443-451 vs 470.
//   * TALL 128x256 (1 / CU): SOFTPLUS_HEAD / MUL / TANGENT where SQ does not apply.
//   * WIDE 256x128 (1 / CU, 32-deep): STORE / SOFTPLUS / RELU / MUL / TANGENT at K % 64 == 0.
//   * T128 128x128 (2 / CU): BWD_SOFTPLUS (its three aux streams need the partner workgroup's main
//     loop to hide: 614 vs 667 us on SQ), first layers (K < 128), edge shapes.
//   bf16 (config C3) tiles: SQ 256x256 (1 / CU, 32-deep) for 128 < N <= 256, else 128x128 / 128x64.
enum LinearTile { LT_BF_SQ, LT_BF_T0, LT_BF_T1, LT_X6_SQ, LT_X6_TALL, LT_X6_WIDE, LT_X6_T128, LT_X6_T1, LT_F_T0_D2,
                  LT_F_T0_D1, LT_F_T1_D2, LT_F_T1_D1 };
#define CN_LINEAR_TILES(X)                 \
    X(LT_BF_SQ, 4, 2, 2, 4, 32, 1, 2, 1)   \
    X(LT_BF_T0, 2, 2, 2, 2, 64, 2, 1, 1)   \
    X(LT_BF_T1, 4, 1, 1, 2, 64, 2, 1, 1)   \
    X(LT_X6_SQ, 4, 2, 2, 4, 16, 1, 2, 2)   \
    X(LT_X6_TALL, 4, 2, 1, 4, 32, 1, 2, 2) \
    X(LT_X6_WIDE, 4, 2, 2, 2, 32, 1, 2, 2) \
    X(LT_X6_T128, 2, 2, 2, 2, 16, 2, 2, 2) \
    X(LT_X6_T1, 4, 1, 1, 2, 16, 2, 2, 2)   \
    X(LT_F_T0_D2, 2, 2, 2, 2, 32, 2, 2, 0) \
    X(LT_F_T0_D1, 2, 2, 2, 2, 32, 2, 1, 0) \
    X(LT_F_T1_D2, 4, 1, 1, 2, 32, 2, 2, 0) \
    X(LT_F_T1_D1, 4, 1, 1, 2, 32, 2, 1, 0)

// measurement build only (-DCN_AB_X6_BWD_SQ=1, profiles/r5_ab.txt): bf16x6 BWD_SOFTPLUS on the 256x256 tile
#ifndef CN_AB_X6_BWD_SQ
#define CN_AB_X6_BWD_SQ 0
#endif

// bf16x6 launches of at most this many rows (the sampler's up-sampling queries: 65,536 rows = one 256x256
// tile per CU, nothing to overlap an epilogue with) take the two-per-CU tiles: SOFTPLUS the 128x128 one,
// SOFTPLUS_HEAD the 128x256 one.  0: off (measurement switch, profiles/r6_ab.txt)
#ifndef CN_X6_SMALL_M
#define CN_X6_SMALL_M 0
#endif

static LinearTile choose_linear_tile(const cn_linear_desc* d) {
    const int e = d->epilogue;
    const bool head = e == CN_EPI_SOFTPLUS_HEAD;
    // one tile spans every column (the 64x128 wave tiles' direct epilogues), no rank-1 term
    const bool wide_n = d->tile == 0 && d->N > 128 && d->N <= 256 && !d->rowv;
    const bool longk = d->K >= 128;  // a first layer's two-chunk main loop cannot hide a 1 / CU epilogue
    if (d->mfma_dtype == CN_MFMA_BF16) {
        // (its LDS-DMA ring prefetches 3 chunks of 32: K >= 96)
        if (wide_n && d->K >= 96 && (longk || head)) return LT_BF_SQ;
        return d->tile == 1 ? LT_BF_T1 : LT_BF_T0;
    }
    if (d->mfma_dtype == CN_MFMA_F32_BF16X6) {
        if (d->tile == 1) return LT_X6_T1;
        if (d->tile == 2) return LT_X6_T128;
        if (d->M <= CN_X6_SMALL_M && wide_n && d->K % 64 == 0 && longk && d->ldb >= 256) {
            if (e == CN_EPI_SOFTPLUS) return LT_X6_T128;
            if (head) return LT_X6_TALL;
        }
        // (BWD_SOFTPLUS on the 256x256 tile: re-measured in round 4 with the branch-free epilogue, equal or
        // slower -- 4.25 vs 4.17 ms per C2 step, profiles/r4_ab.txt r4m)
        if (wide_n && d->K % 32 == 0 && d->ldb >= 256 && (e != CN_EPI_BWD_SOFTPLUS || CN_AB_X6_BWD_SQ) && (longk || head))
            return LT_X6_SQ;
        const bool tall = e == CN_EPI_MUL || e == CN_EPI_TANGENT || head;
        if (d->K % 64 == 0 && tall && d->N > 128 && d->ldb >= 256 && (longk || head)) return LT_X6_TALL;
        // (an aux-reading epilogue with one workgroup per CU no longer overlaps a partner's main loop)
        const bool light = e == CN_EPI_STORE || e == CN_EPI_SOFTPLUS || e == CN_EPI_RELU || e == CN_EPI_MUL ||
                           e == CN_EPI_TANGENT;
        if (d->K % 64 == 0 && light && longk) return LT_X6_WIDE;
        return LT_X6_T128;
    }
    const bool even = (d->K % 64) == 0;  // DEPTH-2 prefetch consumes K in pairs of 32-chunks
    if (d->tile == 1) return even ? LT_F_T1_D2 : LT_F_T1_D1;
    return even ? LT_F_T0_D2 : LT_F_T0_D1;
}

// Validates a descriptor and builds its kernel arguments (a.M == 0: nothing to launch).
static int linear_plan(const cn_linear_desc* d, LinearArgs& a) {
    CN_REQUIRE(d, CN_ERR_ARG, "cn_linear: null desc");
    const bool head = d->epilogue == CN_EPI_SOFTPLUS_HEAD;
    CN_REQUIRE(d->A && d->B && (d->out0 || d->out0_b || head), CN_ERR_ARG, "cn_linear: A, B and out0 (or out0_b) are required");
    CN_REQUIRE(d->M >= 0 && d->N > 0 && d->K > 0, CN_ERR_SHAPE, "cn_linear: bad M/N/K %d/%d/%d", d->M, d->N, d->K);
    CN_REQUIRE(d->mfma_dtype == CN_MFMA_F32 || d->mfma_dtype == CN_MFMA_BF16 || d->mfma_dtype == CN_MFMA_F32_BF16X6,
               CN_ERR_ARG, "cn_linear: bad mfma_dtype %d", d->mfma_dtype);
    const bool bf = d->mfma_dtype == CN_MFMA_BF16;
    const bool x6 = d->mfma_dtype == CN_MFMA_F32_BF16X6;
    CN_REQUIRE(d->K % (bf ? 64 : 32) == 0, CN_ERR_SHAPE, "cn_linear: K=%d must be a multiple of %d", d->K, bf ? 64 : 32);
    CN_REQUIRE(d->tile >= 0 && d->tile <= 2, CN_ERR_ARG, "cn_linear: bad tile %d", d->tile);
    if (x6 && d->a_bf16 && CN_AB_X6_AIMG) {  // (measurement build) A as a bf16x6 term image, rows = lda
        CN_REQUIRE(!d->A2 && !d->aux0_bf16 && !d->aux12_bf16 && !d->out0_b && !d->out1_b && d->lda >= d->M &&
                       al16(d->A) && choose_linear_tile(d) == LT_X6_SQ,
                   CN_ERR_UNSUPPORTED, "cn_linear: bf16x6 A images: 256x256 tile, no A2, lda = image rows >= M");
    } else if (d->a_bf16 || d->aux0_bf16 || d->aux12_bf16 || d->out0_b || d->out1_b) {  // bf16 operand images (ABI v10)
        CN_REQUIRE(bf, CN_ERR_UNSUPPORTED, "cn_linear: bf16 operand images need mfma_dtype CN_MFMA_BF16");
        CN_REQUIRE(!d->a_bf16 || (d->lda % 8 == 0 && (!d->A2 || d->lda2 % 8 == 0)), CN_ERR_ALIGN,
                   "cn_linear: bf16 A / A2 need lda, lda2 multiples of 8");
        const int e = d->epilogue;
        CN_REQUIRE(!d->aux0_bf16 || ((e == CN_EPI_BWD_RELU || e == CN_EPI_MUL || e == CN_EPI_TANGENT ||
                                      e == CN_EPI_BWD_SOFTPLUS) && d->aux0 && !d->rowv && d->ld_aux0 % 8 == 0),
                   CN_ERR_UNSUPPORTED, "cn_linear: a bf16 aux0 is for MUL / TANGENT / BWD_SOFTPLUS / BWD_RELU "
                   "(no rowv, ld_aux0 % 8 == 0)");
        CN_REQUIRE(!d->aux12_bf16 || (e == CN_EPI_BWD_SOFTPLUS && !d->rowv && d->aux1 && d->aux2 &&
                                      d->ld_aux1 % 8 == 0 && d->ld_aux2 % 8 == 0),
                   CN_ERR_UNSUPPORTED, "cn_linear: bf16 aux1 / aux2 are for BWD_SOFTPLUS (both set, no rowv, "
                   "leading dimensions % 8 == 0)");
        // one kernel bit for the epilogue's aux operands: all bf16 or all fp32
        CN_REQUIRE(e != CN_EPI_BWD_SOFTPLUS || !d->aux1 || (d->aux0_bf16 != 0) == (d->aux12_bf16 != 0),
                   CN_ERR_UNSUPPORTED, "cn_linear: BWD_SOFTPLUS's aux0 and aux1 / aux2 are all bf16 images or all fp32");
        CN_REQUIRE(!d->out0_b || (al16(d->out0_b) && d->ld_out0_b % 8 == 0 && d->ld_out0_b < (1 << 20) &&
                                  d->ld_out0_b >= std::max(d->nzero, d->N)),
                   CN_ERR_ALIGN, "cn_linear: out0_b needs 16-byte alignment and ld_out0_b >= nzero, % 8 == 0");
        CN_REQUIRE(!d->out1_b || (d->epilogue == CN_EPI_SOFTPLUS_HEAD && d->colv && d->aux_beta > 0.0f &&
                                  al16(d->out1_b) && d->ld_out1_b % 8 == 0 && d->ld_out1_b < (1 << 20) &&
                                  d->ld_out1_b >= std::max(d->nzero, d->N)),
                   CN_ERR_ARG, "cn_linear: out1_b is SOFTPLUS_HEAD's image of out1 (colv, aux_beta > 0; 16-byte "
                   "aligned, ld % 8 == 0; out1 itself may be NULL)");
    }
    const int K1 = d->A2 ? d->K1 : d->K;
    CN_REQUIRE(K1 > 0 && K1 <= d->K && K1 % (bf ? 64 : 32) == 0, CN_ERR_SHAPE, "cn_linear: bad K1=%d", K1);
    CN_REQUIRE(d->lda >= K1 && d->lda % 4 == 0 && al16(d->A), CN_ERR_ALIGN,
               "cn_linear: A must be 16B aligned with lda>=K1, lda%%4==0");
    if (d->A2) CN_REQUIRE(d->lda2 >= d->K - K1 && d->lda2 % 4 == 0 && al16(d->A2), CN_ERR_ALIGN, "cn_linear: bad A2/lda2");
    const int bn = d->tile == 1 ? 64 : 128;
    if (x6)  // ldb = rows of the chunk-major term image
        CN_REQUIRE(d->ldb >= cdiv(d->N, bn) * bn && al16(d->B), CN_ERR_ALIGN,
                   "cn_linear: bf16x6 B image rows (ldb=%lld) must cover the N tiles", (long long)d->ldb);
    else
        CN_REQUIRE(d->ldb >= d->K && d->ldb % (bf ? 8 : 4) == 0 && al16(d->B), CN_ERR_ALIGN, "cn_linear: bad B/ldb");
    const int nzero = std::max(d->nzero, d->N);
    CN_REQUIRE(nzero <= cdiv(d->N, bn) * bn, CN_ERR_SHAPE,
               "cn_linear: nzero=%d beyond the column tiles covering N=%d (tile width %d)", nzero, d->N, bn);
    CN_REQUIRE(!d->out0 || d->ld_out0 >= nzero, CN_ERR_SHAPE, "cn_linear: ld_out0=%lld < nzero=%d",
               (long long)d->ld_out0, nzero);
    const int e = d->epilogue;
    if (e == CN_EPI_MUL || e == CN_EPI_TANGENT || e == CN_EPI_BWD_SOFTPLUS || e == CN_EPI_BWD_RELU)
        CN_REQUIRE(d->aux0 && d->ld_aux0 >= d->N, CN_ERR_ARG, "cn_linear: epilogue %d needs aux0", e);
    if (e == CN_EPI_MUL || e == CN_EPI_TANGENT || e == CN_EPI_BWD_SOFTPLUS)
        CN_REQUIRE(d->aux_beta > 0.0f, CN_ERR_ARG, "cn_linear: epilogue %d needs aux_beta > 0 (sigma from aux0)", e);
    CN_REQUIRE(d->out1 == nullptr || head, CN_ERR_ARG, "cn_linear: out1 is produced by SOFTPLUS_HEAD only");
    if (head) {
        CN_REQUIRE(d->head_w && d->head_b && d->head_out && !d->rowv && al16(d->head_w), CN_ERR_ARG,
                   "cn_linear: SOFTPLUS_HEAD needs head_w (16B aligned), head_b, head_out and no rowv");
        CN_REQUIRE(d->N <= 256 && (d->odiv == 0.0f || d->odiv == 1.0f), CN_ERR_UNSUPPORTED,
                   "cn_linear: SOFTPLUS_HEAD needs N <= 256 (N=%d) and odiv 1", d->N);
        if (d->out1)
            CN_REQUIRE(d->colv && d->aux_beta > 0.0f && d->ld_out1 >= nzero && al16(d->out1) && d->ld_out1 % 4 == 0,
                       CN_ERR_ARG, "cn_linear: SOFTPLUS_HEAD out1 needs colv, aux_beta > 0 and ld_out1 >= nzero");
    } else {
        CN_REQUIRE(!d->head_out && !d->head_w && !d->head_idx, CN_ERR_ARG, "cn_linear: head_* only for SOFTPLUS_HEAD");
    }
    if (e == CN_EPI_BWD_SOFTPLUS)
        CN_REQUIRE((d->aux1 == nullptr) == (d->aux2 == nullptr) &&
                       (!d->aux1 || (d->ld_aux1 >= d->N && d->ld_aux2 >= d->N)),
                   CN_ERR_ARG, "cn_linear: BWD_SOFTPLUS takes aux1 (s) and aux2 (u') together");
    else
        CN_REQUIRE(d->aux1 == nullptr && d->aux2 == nullptr, CN_ERR_ARG, "cn_linear: aux1/aux2 only for BWD_SOFTPLUS");
    if (e == CN_EPI_MUL && d->nsplit < d->N)
        CN_REQUIRE(d->out_split && d->nsplit >= 0 && d->ld_split >= d->N - d->nsplit, CN_ERR_ARG,
                   "cn_linear: split output required");
    CN_REQUIRE((d->rowv == nullptr) == (d->colv == nullptr) || head, CN_ERR_ARG, "cn_linear: rowv/colv go together");
    CN_REQUIRE(al16(d->bias) && al16(d->colv), CN_ERR_ALIGN, "cn_linear: bias / colv must be 16-byte aligned");
    CN_REQUIRE((!d->bias && !d->colv) || d->N <= kTblCols, CN_ERR_UNSUPPORTED,
               "cn_linear: N=%d > %d with a bias / colv", d->N, kTblCols);
    // the epilogue moves 4 columns per 16-byte access
    CN_REQUIRE(d->N % 4 == 0 && nzero % 4 == 0 && (e != CN_EPI_MUL || d->nsplit % 4 == 0), CN_ERR_SHAPE,
               "cn_linear: N, nzero and nsplit must be multiples of 4");
    CN_REQUIRE(al16(d->out0) && d->ld_out0 % 4 == 0 && (!d->out1 || (al16(d->out1) && d->ld_out1 % 4 == 0)) &&
                   (!d->aux0 || (al16(d->aux0) && d->ld_aux0 % 4 == 0)) &&
                   (!d->aux1 || (al16(d->aux1) && d->ld_aux1 % 4 == 0)) &&
                   (!d->aux2 || (al16(d->aux2) && d->ld_aux2 % 4 == 0)) &&
                   (!d->out_split || (al16(d->out_split) && d->ld_split % 4 == 0)),
               CN_ERR_ALIGN, "cn_linear: outputs / aux must be 16-byte aligned with leading dims % 4 == 0");
    // buffer views address a 128-row tile with 32-bit byte offsets
    constexpr int64_t kMaxLd = 1 << 20;
    CN_REQUIRE(d->lda < kMaxLd && d->lda2 < kMaxLd && d->ldb < kMaxLd && d->ld_aux0 < kMaxLd && d->ld_aux1 < kMaxLd && d->ld_aux2 < kMaxLd &&
                   d->ld_out0 < kMaxLd && d->ld_out1 < kMaxLd && d->ld_split < kMaxLd,
               CN_ERR_SHAPE, "cn_linear: leading dimensions must be < 2^20");
    a = LinearArgs{};
    a.A = static_cast<const float*>(d->A); a.A2 = static_cast<const float*>(d->A2); a.B = d->B;
    a.bias = d->bias; a.rowv = d->rowv; a.colv = d->colv;
    a.aux0 = static_cast<const float*>(d->aux0); a.aux1 = d->aux1; a.aux2 = d->aux2;
    a.out0 = d->out0; a.out1 = d->out1; a.out_split = d->out_split;
    a.lda = (int)d->lda; a.lda2 = (int)d->lda2; a.ldb = (int)d->ldb;
    a.ld_aux0 = (int)d->ld_aux0; a.ld_aux1 = (int)d->ld_aux1; a.ld_aux2 = (int)d->ld_aux2;
    a.aux_c = -d->aux_beta * 1.44269504088896341f;
    a.aux2_scale = d->aux2_scale;
    a.head_w = d->head_w; a.head_b = d->head_b; a.head_out = d->head_out; a.head_idx = d->head_idx;
    a.flags = d->flags;
    a.ld_out0 = (int)d->ld_out0; a.ld_out1 = (int)d->ld_out1; a.ld_split = (int)d->ld_split;
    a.M = d->M; a.N = d->N; a.K = d->K; a.K1 = K1; a.nzero = nzero;
    a.nsplit = (e == CN_EPI_MUL && d->out_split) ? d->nsplit : d->N;
    const float adiv = d->adiv == 0.0f ? 1.0f : d->adiv;
    const float odiv = d->odiv == 0.0f ? 1.0f : d->odiv;
    a.inv_adiv = 1.0f / adiv;
    a.inv_odiv = 1.0f / odiv;
    a.beta = d->beta;
    a.threshold = d->threshold;
    a.out0_b = static_cast<bf16_t*>(d->out0_b);
    a.out1_b = static_cast<bf16_t*>(d->out1_b);
    a.ld_out0_b = (int)d->ld_out0_b;
    a.ld_out1_b = (int)d->ld_out1_b;
    return CN_OK;
}

extern "C" int cn_linear(const cn_linear_desc* d, cn_stream_t stream) {
    LinearArgs a;
    int rc = linear_plan(d, a);
    if (rc || d->M == 0) return rc;
    hipStream_t s = (hipStream_t)stream;
    switch (choose_linear_tile(d)) {
#define CN_TILE_CASE(T, WM, WN, TM, TN, BK, OCC, DEPTH, MODE) \
        case T: return launch_linear_tile<WM, WN, TM, TN, BK, OCC, DEPTH, MODE>(d, a, s);
        CN_LINEAR_TILES(CN_TILE_CASE)
#undef CN_TILE_CASE
    }
    set_error("cn_linear: no tile");
    return CN_ERR_UNSUPPORTED;
}

extern "C" int cn_linear_kernel_name(const cn_linear_desc* d, char* buf, int32_t len) {
    CN_REQUIRE(d && buf && len > 0, CN_ERR_ARG, "cn_linear_kernel_name: null desc / buffer");
    const char* args = "";
    int mode = 0;
    switch (choose_linear_tile(d)) {
#define CN_TILE_NAME(T, WM, WN, TM, TN, BK, OCC, DEPTH, MODE) \
        case T: args = #WM ", " #WN ", " #TM ", " #TN ", " #BK ", " #OCC ", " #DEPTH; mode = linear_mode_bits(d, MODE); break;
        CN_LINEAR_TILES(CN_TILE_NAME)
#undef CN_TILE_NAME
    }
    const int n = snprintf(buf, (size_t)len, "void cn::linear_kernel<%s, %d, %s, %d>(cn::LinearArgs)", args,
                           d->epilogue, d->rowv && (mode & 8) == 0 ? "true" : "false", mode);
    CN_REQUIRE(n < len, CN_ERR_SHAPE, "cn_linear_kernel_name: buffer of %d bytes too small (%d)", len, n + 1);
    return n;
}


extern "C" int cn_row_head(int32_t M, int32_t K, const float* A, int64_t lda, const float* W, int64_t ldw,
                           const float* b, int32_t C, int32_t act, float* out, int64_t ld_out,
                           const int32_t* dst_index, cn_stream_t stream) {
    CN_REQUIRE(A && W && out, CN_ERR_ARG, "cn_row_head: null pointer");
    CN_REQUIRE(K > 0 && K <= 256 && K % 4 == 0 && C >= 1 && C <= 4, CN_ERR_UNSUPPORTED, "cn_row_head: K=%d C=%d", K, C);
    CN_REQUIRE(lda % 4 == 0 && ldw % 4 == 0 && al16(A) && al16(W), CN_ERR_ALIGN, "cn_row_head: alignment");
    CN_REQUIRE(act == 0 || act == 1, CN_ERR_ARG, "cn_row_head: act");
    if (M == 0) return CN_OK;
    const int blocks = std::min(cdiv(M, 32), 8192);  // 4 waves x 8 rows per iteration
    row_head_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(M, K, A, lda, W, ldw, b, C, act, out, ld_out, dst_index);
    return check_launch("cn_row_head");
}

extern "C" int cn_scale_cols(int32_t M, int32_t N, const float* X, int64_t ldx, const float* w, const float* rowv,
                             float* out, int64_t ld_out, float act_beta, cn_stream_t stream) {
    CN_REQUIRE(act_beta >= 0.0f, CN_ERR_ARG, "cn_scale_cols: act_beta must be >= 0");
    CN_REQUIRE(X && w && out, CN_ERR_ARG, "cn_scale_cols: null pointer");
    CN_REQUIRE(N % 4 == 0 && ldx % 4 == 0 && ld_out % 4 == 0 && al16(X) && al16(w) && al16(out), CN_ERR_ALIGN,
               "cn_scale_cols: N, leading dimensions and pointers must be multiples of 4 floats");
    if ((int64_t)M * N == 0) return CN_OK;
    const int64_t tot = (int64_t)M * (N / 4);
    const int blocks = (int)std::min<int64_t>((tot + 255) / 256, 8192);
    scale_cols_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(M, N / 4, X, ldx, w, rowv, out, ld_out,
                                                               -act_beta * 1.44269504088896341f);
    return check_launch("cn_scale_cols");
}

extern "C" size_t cn_softplus_adjoint_workspace_bytes(int32_t M, int32_t N) {
    return sizeof(float) * (size_t)std::max(1, cdiv(M, kSaRows)) * (std::max(N, 4) + 1);
}

extern "C" int cn_softplus_adjoint(int32_t M, int32_t N, const void* D, int64_t ldd, const void* act, int64_t lda,
                                   float act_beta, const float* rowv, const float* colv, const void* aux1,
                                   int64_t ld1, const void* aux2, int64_t ld2, float aux2_scale, void* out,
                                   int64_t ld_out, int32_t out_bf16, int32_t in_bf16, float* cs_out, float* rs_out,
                                   float cs_div, float* workspace, int64_t workspace_bytes, cn_stream_t stream) {
    CN_REQUIRE(act && out && act_beta > 0.0f, CN_ERR_ARG, "cn_softplus_adjoint: act, out and act_beta > 0 required");
    CN_REQUIRE((rowv == nullptr) == (colv == nullptr) && (aux1 == nullptr) == (aux2 == nullptr), CN_ERR_ARG,
               "cn_softplus_adjoint: rowv/colv and aux1/aux2 go together");
    CN_REQUIRE(in_bf16 >= 0 && in_bf16 < 8, CN_ERR_ARG, "cn_softplus_adjoint: in_bf16 is a 3-bit mask");
    CN_REQUIRE(N % 4 == 0 && lda % 4 == 0 && ld_out % 4 == 0 && al8(act) && al8(out) &&
                   (!D || (ldd % 4 == 0 && al8(D))) && (!colv || al16(colv)) &&
                   (!aux1 || (ld1 % 4 == 0 && ld2 % 4 == 0 && al8(aux1) && al8(aux2))) &&
                   ((in_bf16 & 2) || al16(act)) && (out_bf16 || al16(out)) && (!D || (in_bf16 & 1) || al16(D)) &&
                   (!aux1 || (in_bf16 & 4) || (al16(aux1) && al16(aux2))),
               CN_ERR_ALIGN, "cn_softplus_adjoint: N, leading dimensions and pointers must be multiples of 4 floats");
    if (cs_out) {
        CN_REQUIRE(N >= 4 && N <= 1024 && workspace &&
                       (size_t)workspace_bytes >= cn_softplus_adjoint_workspace_bytes(M, N),
                   CN_ERR_SHAPE, "cn_softplus_adjoint: column sums need N <= 1024 and the workspace");
        if (M == 0) {
            // no rows: zero sums (one reduction launch for both)
            return launch_slab_jobs(slab_job(workspace, 0, N, 1, N, N, cs_out, N, 1.0f, 0),
                                    rs_out ? slab_job(workspace, 0, 1, 1, 1, 1, rs_out, 1, 1.0f, 0) : SlabJob{},
                                    (hipStream_t)stream);
        }
        const int nblk = cdiv(M, kSaRows);
        hipStream_t s = (hipStream_t)stream;
        float* rpart = rs_out ? workspace + (size_t)nblk * N : nullptr;
        switch (in_bf16) {
#define CN_SA_CS(IB)                                                                                             \
            case IB:                                                                                             \
                softplus_adjoint_cs_kernel<IB><<<nblk, 256, 0, s>>>(M, N / 4, D, ldd, act, lda,                   \
                                                                    -act_beta * 1.44269504088896341f, rowv, colv, \
                                                                    aux1, ld1, aux2, ld2, aux2_scale, out, ld_out, \
                                                                    out_bf16 != 0, workspace, rpart);            \
                break;
            CN_SA_CS(0) CN_SA_CS(1) CN_SA_CS(2) CN_SA_CS(3) CN_SA_CS(4) CN_SA_CS(5) CN_SA_CS(6) CN_SA_CS(7)
#undef CN_SA_CS
        }
        int rc = check_launch("cn_softplus_adjoint");
        if (rc) return rc;
        const float dv = cs_div == 0.f ? 1.f : cs_div;
        return launch_slab_jobs(slab_job(workspace, nblk, N, 1, N, N, cs_out, N, dv, 0),
                                rs_out ? slab_job(rpart, nblk, 1, 1, 1, 1, rs_out, 1, dv, 0) : SlabJob{}, s);
    }
    if ((int64_t)M * N == 0) return CN_OK;
    const int64_t tot = (int64_t)M * (N / 4);
    const int blocks = (int)std::min<int64_t>((tot + 255) / 256, 8192);
    switch (in_bf16) {
#define CN_SA(IB)                                                                                                \
        case IB:                                                                                                 \
            softplus_adjoint_kernel<IB><<<blocks, 256, 0, (hipStream_t)stream>>>(                                \
                M, N / 4, D, ldd, act, lda, -act_beta * 1.44269504088896341f, rowv, colv, aux1, ld1, aux2, ld2,  \
                aux2_scale, out, ld_out, out_bf16 != 0);                                                         \
            break;
        CN_SA(0) CN_SA(1) CN_SA(2) CN_SA(3) CN_SA(4) CN_SA(5) CN_SA(6) CN_SA(7)
#undef CN_SA
    }
    return check_launch("cn_softplus_adjoint");
}

extern "C" size_t cn_rgb_head_bwd_workspace_bytes(int32_t M, int32_t K) {
    return sizeof(float) * (size_t)std::max(1, cdiv(M, kHeadRowsPerBlock)) * 4 * K;
}

extern "C" int cn_rgb_head_bwd(int32_t M, int32_t K, const float* drgb, const float* rgb, const float* H3,
                               int64_t ld_h, const float* W3, void* dZ2, int64_t ld_dz, int32_t dz_bf16, float* dW3,
                               float* db3, float* workspace, int64_t workspace_bytes, cn_stream_t stream) {
    CN_REQUIRE(drgb && rgb && H3 && W3 && dZ2 && dW3 && db3 && workspace, CN_ERR_ARG, "cn_rgb_head_bwd: null pointer");
    CN_REQUIRE(K > 0 && K <= 256, CN_ERR_UNSUPPORTED, "cn_rgb_head_bwd: K=%d", K);
    CN_REQUIRE(K % 4 == 0 && ld_h % 4 == 0 && ld_dz % 4 == 0 && al16(H3) && (dz_bf16 ? al8(dZ2) : al16(dZ2)) && al16(W3), CN_ERR_ALIGN,
               "cn_rgb_head_bwd: K, leading dimensions and H3 / dZ2 / W3 must be multiples of 4 floats");
    CN_REQUIRE((size_t)workspace_bytes >= cn_rgb_head_bwd_workspace_bytes(M, K), CN_ERR_SHAPE, "cn_rgb_head_bwd: workspace");
    const int nblk = std::max(1, cdiv(M, kHeadRowsPerBlock));
    hipStream_t s = (hipStream_t)stream;
    rgb_head_bwd_kernel<<<nblk, 256, 0, s>>>(M, K, drgb, rgb, H3, ld_h, W3, dZ2, ld_dz, dz_bf16 != 0, workspace);
    int rc = check_launch("cn_rgb_head_bwd");
    if (rc) return rc;
    return launch_slab_jobs(slab_job(workspace, nblk, 4 * K, 3, K, K, dW3, K, 1.0f, 0),
                            slab_job(workspace + 3 * K, nblk, 4 * K, 1, 3, 3, db3, 3, 1.0f, 0), s);
}

extern "C" size_t cn_colsum_workspace_bytes(int32_t M, int32_t K) {
    return sizeof(float) * (size_t)std::max(1, cdiv(M, kColsumRows)) * K;
}

extern "C" int cn_colsum(int32_t M, int32_t K, const float* w, const float* X, int64_t ldx, float wdiv, float* out,
                         int32_t accumulate, float* workspace, int64_t workspace_bytes, cn_stream_t stream) {
    CN_REQUIRE(X && out && workspace, CN_ERR_ARG, "cn_colsum: null pointer");
    CN_REQUIRE(K > 0 && ldx >= K, CN_ERR_SHAPE, "cn_colsum: K=%d ldx=%lld", K, (long long)ldx);
    CN_REQUIRE((size_t)workspace_bytes >= cn_colsum_workspace_bytes(M, K), CN_ERR_SHAPE, "cn_colsum: workspace");
    const int nblk = std::max(1, cdiv(M, kColsumRows));
    hipStream_t s = (hipStream_t)stream;
    dim3 grid(nblk, cdiv(K, 256));
    if (M > 0) {
        colsum_kernel<<<grid, 256, 0, s>>>(M, K, w, X, ldx, workspace);
        int rc = check_launch("cn_colsum");
        if (rc) return rc;
    } else {
        if (hipMemsetAsync(workspace, 0, sizeof(float) * K, s) != hipSuccess) {
            set_error("cn_colsum: hipMemsetAsync failed");
            return CN_ERR_LAUNCH;
        }
    }
    return launch_slab_reduce(workspace, nblk, K, 1, K, K, out, K, wdiv == 0.f ? 1.f : wdiv, accumulate, s);
}
