// cn_wgrad.hip — weight gradients dW = Σ_m Yᵀ X (+ a second pair) and db = Σ_m Y over the M sample
// rows (the reduction of every Linear's backward, model/neus_fields.py:273-303, 364-373), split
// over workgroups into fp32 slabs that slab_reduce_kernel sums in a fixed order (bitwise
// reproducible, no atomics).
#include "cn_mfma.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>


namespace cn {

// ---------------------------------------------------------------------------
// Weight gradient.
struct WgradArgs {
    const float* Y0;
    const float* X0;
    const float* Y1;
    const float* X1;
    float* part;   // [nslices][Npad][Kpad]
    float* bpart;  // [nslices][Npad]
    int ldy0, ldx0, ldy1, ldx1;
    int M, Npad, Kpad, npairs, rows_per_slice, n_tiles_n, n_tiles_k, nslices;
    int yb, xb;  // wgrad_b16r_kernel: the Y / X side are bf16 operand images
};

// Several independent weight gradients in one launch of the stage-ring kernel (cn_wgrad_batch):
// job i takes the next blocks[i] workgroups, each job its own M-slices and slabs.
constexpr int kWgradBatchMax = 16;
struct WgradBatch {
    WgradArgs job[kWgradBatchMax];
    int blocks[kWgradBatchMax];
    int njobs;
};

template <int WM, int WN, int TM, int TN>
__global__ void __launch_bounds__(64 * WM * WN, 2) wgrad_kernel(WgradArgs p) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BNo = 32 * TM * WM;  // output rows (n) per tile
    constexpr int BKo = 32 * TN * WN;  // output cols (k) per tile
    constexpr int MC = 32;             // sample rows per chunk
    constexpr int YF4 = MC * BNo / 4;
    constexpr int XF4 = MC * BKo / 4;
    static_assert(YF4 % NT == 0 && XF4 % NT == 0, "tile/thread mismatch");
    constexpr int YLD = YF4 / NT;
    constexpr int XLD = XF4 / NT;

    __shared__ __attribute__((aligned(16))) float smem[2 * MC * (BNo + BKo)];
    float* sY = smem;
    float* sX = smem + 2 * MC * BNo;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;

    // XCD-aware: blocks b and b+8 share an XCD (and its L2), so the T output tiles
    // of one M-slice, which read the same Y / X rows, are placed 8 blocks apart
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int b = blockIdx.x;
    const int tile = (b >> 3) % T;
    const int slice = (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;
    const int tn = tile / p.n_tiles_k;
    const int tk = tile % p.n_tiles_k;
    const int n0 = tn * BNo;
    const int k0 = tk * BKo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = (tk == 0) && (p.bpart != nullptr);

    // buffer views (see linear_kernel): the chunk's first row is the descriptor
    // base (SALU), rows past mend read as zero through the range check
    constexpr int YRS = NT / (BNo / 4);  // staged rows per Y load instruction
    constexpr int XRS = NT / (BKo / 4);
    const int yrow = tid / (BNo / 4), yc4 = tid % (BNo / 4);
    const int xrow = tid / (BKo / 4), xc4 = tid % (BKo / 4);
    floatx4 ry[YLD], rx[XLD];
    auto gload = [&](int c) {
        const int pair = c >= nch;
        const int mrow = mbeg + (c - pair * nch) * MC;
        const float* Y = pair ? p.Y1 : p.Y0;
        const float* X = pair ? p.X1 : p.X0;
        const int ly = pair ? p.ldy1 : p.ldy0;
        const int lx = pair ? p.ldx1 : p.ldx0;
        const int nrows = min(MC, mend - mrow);
        const rsrc_t vY = make_view(Y + (int64_t)mrow * ly + n0, (nrows * ly - n0) * 4);
        const rsrc_t vX = make_view(X + (int64_t)mrow * lx + k0, (nrows * lx - k0) * 4);
#pragma unroll
        for (int q = 0; q < YLD; ++q) ry[q] = bload4(vY, ((yrow + q * YRS) * ly + yc4 * 4) * 4, 0);
#pragma unroll
        for (int q = 0; q < XLD; ++q) rx[q] = bload4(vX, ((xrow + q * XRS) * lx + xc4 * 4) * 4, 0);
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int q = 0; q < YLD; ++q) {
            const int f = tid + q * NT;
            *reinterpret_cast<floatx4*>(sY + buf * MC * BNo + f * 4) = ry[q];
        }
#pragma unroll
        for (int q = 0; q < XLD; ++q) {
            const int f = tid + q * NT;
            *reinterpret_cast<floatx4*>(sX + buf * MC * BKo + f * 4) = rx[q];
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    float bacc = 0.0f;

    if (total > 0) {
        gload(0);
        lstore(0);
    }
    __syncthreads();
    const int h = lane >> 5;
    const int ycol = wm * TM * 32 + (lane & 31);
    const int xcol = wn * TN * 32 + (lane & 31);
    for (int c = 0; c < total; ++c) {
        const int cur = c & 1;
        if (c + 1 < total) gload(c + 1);
        const float* yb = sY + cur * MC * BNo;
        const float* xb = sX + cur * MC * BKo;
        if (do_bias && c < nch && tid < BNo) {
#pragma unroll 8
            for (int r = 0; r < MC; ++r) bacc += yb[r * BNo + tid];
        }
#pragma unroll
        for (int s = 0; s < MC / 2; ++s) {
            float af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = yb[(2 * s + h) * BNo + ycol + i * 32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = xb[(2 * s + h) * BKo + xcol + j * 32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (c + 1 < total) lstore(cur ^ 1);
        __syncthreads();
    }

    // slab stores: lane offset in voffset, the accumulator row step in soffset
    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = k0 + wn * TN * 32 + j * 32 + (lane & 31);
            const int rbase = n0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
            const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[i][j][r]);
        }
    }
    if (do_bias && tid < BNo) p.bpart[(int64_t)slice * p.Npad + n0 + tid] = bacc;
}

// bf16-operand weight gradient (config C3): the same tiles and slabs as
// wgrad_kernel, with Y and X rounded to bf16 while staging and written
// TRANSPOSED into LDS ([n][m] and [k][m], 64 m per row + 8 pad = 36 dwords), so
// one ds_read_b128 gives a lane the 8 consecutive m of its
// v_mfma_f32_32x32x16_bf16 fragment.  A thread stages 4 rows x 4 columns per
// pass and packs each column's 4 m into one ds_write_b64; the 16-byte blocks of
// a row are XOR-swizzled so those writes do not collide on banks.  db is summed from the
// fp32 values in registers (partials reduced through LDS at the end).
template <int WM, int WN, int TM, int TN>
__global__ void __launch_bounds__(64 * WM * WN, 2) wgrad_bf16_kernel(WgradArgs p) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BNo = 32 * TM * WM;
    constexpr int BKo = 32 * TN * WN;
    constexpr int MC = 64;
    constexpr int LSB = MC / 2 + 4;  // dwords per LDS row
    constexpr int YC = BNo / 4, XC = BKo / 4;        // float4 column groups per staged row
    constexpr int YMQ = NT / YC, XMQ = NT / XC;      // m-quads per pass
    constexpr int YP = (MC / 4) / YMQ, XP = (MC / 4) / XMQ;
    static_assert(YP >= 1 && XP >= 1 && YMQ * YC == NT && XMQ * XC == NT, "staging geometry");
    static_assert(2 * BNo <= (BNo + BKo) * LSB, "bias partials fit in LDS");

    __shared__ __attribute__((aligned(16))) float smem[2 * (BNo + BKo) * LSB];
    float* sY = smem;
    float* sX = smem + 2 * BNo * LSB;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int b = blockIdx.x;
    const int tile = (b >> 3) % T;
    const int slice = (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;
    const int tn = tile / p.n_tiles_k;
    const int tk = tile % p.n_tiles_k;
    const int n0 = tn * BNo;
    const int k0 = tk * BKo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = (tk == 0) && (p.bpart != nullptr);

    const int yc = tid % YC, ymq = tid / YC;
    const int xc = tid % XC, xmq = tid / XC;
    floatx4 ry[YP][4], rx[XP][4];
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    auto gload = [&](int c) {
        const int pair = c >= nch;
        const int mrow = mbeg + (c - pair * nch) * MC;
        const float* Y = pair ? p.Y1 : p.Y0;
        const float* X = pair ? p.X1 : p.X0;
        const int ly = pair ? p.ldy1 : p.ldy0;
        const int lx = pair ? p.ldx1 : p.ldx0;
        const int nrows = min(MC, mend - mrow);
        const rsrc_t vY = make_view(Y + (int64_t)mrow * ly + n0, (nrows * ly - n0) * 4);
        const rsrc_t vX = make_view(X + (int64_t)mrow * lx + k0, (nrows * lx - k0) * 4);
#pragma unroll
        for (int pp = 0; pp < YP; ++pp)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                ry[pp][r] = bload4(vY, (((ymq + pp * YMQ) * 4 + r) * ly + yc * 4) * 4, 0);
#pragma unroll
        for (int pp = 0; pp < XP; ++pp)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                rx[pp][r] = bload4(vX, (((xmq + pp * XMQ) * 4 + r) * lx + xc * 4) * 4, 0);
    };
    // XOR swizzle of the 16-byte blocks of a row by (row >> 2) & 7: the staging
    // writes (threads on rows 4 apart) spread over all banks; reads undo it
    auto swz = [&](int row, int mq) { return row * LSB + (((mq >> 1) ^ ((row >> 2) & 7)) << 2) + ((mq & 1) << 1); };
    auto lstore = [&](int buf, bool bias) {
        float* y = sY + buf * BNo * LSB;
        float* x = sX + buf * BKo * LSB;
#pragma unroll
        for (int pp = 0; pp < YP; ++pp)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const floatx4 col = {ry[pp][0][e], ry[pp][1][e], ry[pp][2][e], ry[pp][3][e]};
                if (bias) bsum[e] += (col[0] + col[1]) + (col[2] + col[3]);
                *reinterpret_cast<bf16x4*>(y + swz(yc * 4 + e, ymq + pp * YMQ)) = __builtin_convertvector(col, bf16x4);
            }
#pragma unroll
        for (int pp = 0; pp < XP; ++pp)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const floatx4 col = {rx[pp][0][e], rx[pp][1][e], rx[pp][2][e], rx[pp][3][e]};
                *reinterpret_cast<bf16x4*>(x + swz(xc * 4 + e, xmq + pp * XMQ)) = __builtin_convertvector(col, bf16x4);
            }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    if (total > 0) {
        gload(0);
        lstore(0, do_bias && nch > 0);
    }
    __syncthreads();
    const int h = lane >> 5;
    const int ycol = wm * TM * 32 + (lane & 31);
    const int xcol = wn * TN * 32 + (lane & 31);
    for (int c = 0; c < total; ++c) {
        const int cur = c & 1;
        const bool more = c + 1 < total;
        if (more) gload(c + 1);
        const float* yb = sY + cur * BNo * LSB + ycol * LSB;
        const float* xb = sX + cur * BKo * LSB + xcol * LSB;
        const int sw = ((lane & 31) >> 2) & 7;  // (row >> 2) & 7 of this lane's rows
#pragma unroll
        for (int ks = 0; ks < MC / 16; ++ks) {
            const int blk = ((2 * ks + h) ^ sw) << 2;
            bf16x8 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(yb + i * 32 * LSB + blk);
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const bf16x8*>(xb + j * 32 * LSB + blk);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (more) lstore(cur ^ 1, do_bias && c + 1 < nch);
        __syncthreads();
    }

    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = k0 + wn * TN * 32 + j * 32 + (lane & 31);
            const int rbase = n0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
            const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[i][j][r]);
        }
    }
    if (do_bias) {  // reduce the per-thread column partials over the m-quads (fixed order)
        float* red = smem;  // [YMQ][BNo]
#pragma unroll
        for (int e = 0; e < 4; ++e) red[ymq * BNo + yc * 4 + e] = bsum[e];
        __syncthreads();
        if (tid < BNo) {
            float t = 0.0f;
            for (int q = 0; q < YMQ; ++q) t += red[q * BNo + tid];
            p.bpart[(int64_t)slice * p.Npad + n0 + tid] = t;
        }
    }
}

// fp32 weight gradient on the bf16 MFMA (CN_MFMA_F32_BF16X6), 128x128 output
// tiles: Y and X are split into three bf16 terms while staging (split3) and the
// six term products with i + j <= 2 accumulate in fp32, as in linear_kernel
// MODE 2.  Staging is transposed like wgrad_bf16_kernel's, 32 sample rows per
// chunk: thread t holds m-quad t % 8 of column group t / 8 (4 m x 4 columns of
// Y and of X), so 16 contiguous lanes write two LDS rows 4 apart whose 64-byte
// segments fall on the two halves of the 32 write banks; an LDS row is the three
// 16-dword term planes + 4 pad (52 dwords: the ds_read_b128 fragment reads of 16
// consecutive rows hit 16 distinct bank quads).  One LDS buffer (53 KB, two
// workgroups per CU): the next chunk's loads fly during the MFMAs.  TN = 1: 64
// output columns, X staged by the first two waves.  WM = 4, TN = 4: a whole
// 256x256 layer per workgroup of 8 waves (one per CU, 106 KB LDS): every staged
// element feeds twice the MFMA work of the 128x128 tile.
template <int WM, int TN>
__global__ void __launch_bounds__(128 * WM, 2) wgrad_x6_kernel(WgradArgs p) {
    constexpr int TM = 2, WN = 2, NT = 128 * WM;
    constexpr int BNo = 64 * WM, BKo = 64 * TN, MC = 32, MQ = MC / 4;
    constexpr int PL = MC / 2;       // dwords per term plane of a row
    constexpr int LSB = 3 * PL + 4;  // 52
    constexpr int XT = MQ * (BKo / 4);  // threads staging X (256 or 128: whole waves)
    static_assert(MQ * (BNo / 4) == NT && XT <= NT && XT % 64 == 0, "staging geometry: whole waves");
    static_assert(MQ * BNo <= (BNo + BKo) * LSB, "bias partials fit in LDS");
    __shared__ __attribute__((aligned(16))) float smem[(BNo + BKo) * LSB];
    float* sY = smem;
    float* sX = smem + BNo * LSB;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int b = blockIdx.x;
    const int tile = (b >> 3) % T;
    const int slice = (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;
    const int tn = tile / p.n_tiles_k;
    const int tk = tile % p.n_tiles_k;
    const int n0 = tn * BNo;
    const int k0 = tk * BKo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = (tk == 0) && (p.bpart != nullptr);

    const int mq = tid % MQ, cg = tid / MQ;
    floatx4 ry[4], rx[4];
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    auto gload = [&](int c) {
        const int pair = c >= nch;
        const int mrow = mbeg + (c - pair * nch) * MC;
        const float* Y = pair ? p.Y1 : p.Y0;
        const float* X = pair ? p.X1 : p.X0;
        const int ly = pair ? p.ldy1 : p.ldy0;
        const int lx = pair ? p.ldx1 : p.ldx0;
        const int nrows = min(MC, mend - mrow);
        const rsrc_t vY = make_view(Y + (int64_t)mrow * ly + n0, (nrows * ly - n0) * 4);
        const rsrc_t vX = make_view(X + (int64_t)mrow * lx + k0, (nrows * lx - k0) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) ry[r] = bload4(vY, ((mq * 4 + r) * ly + cg * 4) * 4, 0);
        if (XT == NT || tid < XT) {
#pragma unroll
            for (int r = 0; r < 4; ++r) rx[r] = bload4(vX, ((mq * 4 + r) * lx + cg * 4) * 4, 0);
        }
    };
    auto lstore = [&](bool bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const floatx4 col = {ry[0][e], ry[1][e], ry[2][e], ry[3][e]};
            if (bias) bsum[e] += (col[0] + col[1]) + (col[2] + col[3]);
            bf16x4 t0, t1, t2;
            split3(col, t0, t1, t2);
            float* y = sY + (cg * 4 + e) * LSB + mq * 2;
            *reinterpret_cast<bf16x4*>(y) = t0;
            *reinterpret_cast<bf16x4*>(y + PL) = t1;
            *reinterpret_cast<bf16x4*>(y + 2 * PL) = t2;
        }
        if (XT < NT && tid >= XT) return;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const floatx4 col = {rx[0][e], rx[1][e], rx[2][e], rx[3][e]};
            bf16x4 t0, t1, t2;
            split3(col, t0, t1, t2);
            float* x = sX + (cg * 4 + e) * LSB + mq * 2;
            *reinterpret_cast<bf16x4*>(x) = t0;
            *reinterpret_cast<bf16x4*>(x + PL) = t1;
            *reinterpret_cast<bf16x4*>(x + 2 * PL) = t2;
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    const int h = lane >> 5;
    const float* yb = sY + (wm * TM * 32 + (lane & 31)) * LSB + 4 * h;
    const float* xb = sX + (wn * TN * 32 + (lane & 31)) * LSB + 4 * h;
    if (total > 0) gload(0);
    for (int c = 0; c < total; ++c) {
        if (c > 0) __syncthreads();  // the previous chunk's fragment reads are done
        lstore(do_bias && c < nch);
        __syncthreads();
        if (c + 1 < total) gload(c + 1);
#pragma unroll
        for (int ks = 0; ks < MC / 16; ++ks) {
            bf16x8 af[3][TM], bf[3][TN];
#pragma unroll
            for (int t = 0; t < 3; ++t) {
#pragma unroll
                for (int i = 0; i < TM; ++i) af[t][i] = *reinterpret_cast<const bf16x8*>(yb + i * 32 * LSB + t * PL + ks * 8);
#pragma unroll
                for (int j = 0; j < TN; ++j) bf[t][j] = *reinterpret_cast<const bf16x8*>(xb + j * 32 * LSB + t * PL + ks * 8);
            }
            constexpr int TA[6] = {0, 1, 0, 2, 1, 0};
            constexpr int TB[6] = {0, 0, 1, 0, 1, 2};
#pragma unroll
            for (int u = 0; u < 6; ++u)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[TA[u]][i], bf[TB[u]][j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();  // LDS is reused for the bias partials

    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = k0 + wn * TN * 32 + j * 32 + (lane & 31);
            const int rbase = n0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
            const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[i][j][r]);
        }
    }
    if (do_bias) {  // reduce the per-thread column partials over the m-quads (fixed order)
        float* red = smem;  // [MQ][BNo]
#pragma unroll
        for (int e = 0; e < 4; ++e) red[mq * BNo + cg * 4 + e] = bsum[e];
        __syncthreads();
        if (tid < BNo) {
            float t = 0.0f;
            for (int q = 0; q < MQ; ++q) t += red[q * BNo + tid];
            p.bpart[(int64_t)slice * p.Npad + n0 + tid] = t;
        }
    }
}

// Whole-layer (256x256) bf16x6 weight gradient on a stage ring: 16 sample rows per stage,
// two split-image buffers (2 x 56 KB: rows of 3 term planes x 8 dwords + 4 pad, reads
// conflict-free, staging writes 2-way) and NRAW register sets of raw fp32 rows, so ONE
// barrier separates consecutive stages and everything else of stage c+1 -- the global
// loads of stage c+NRAW, the bf16 split and the LDS writes of stage c+1 into the free
// buffer -- sits in the same basic block as stage c's 48 MFMAs per wave.  The stage is four
// segments pinned by sched_barrier (column block j's 12 MFMAs beside split column j), so
// the scheduler interleaves each segment's split VALU and LDS writes with its MFMAs: in
// the same wave's stream they fill MFMA issue gaps (a partner wave's VALU does not,
// tools/probes/mfma_bf16_valu_probe.hip; sched_group_barrier patterns were not followed).
// Waves 0-3 stage Y, waves 4-7 stage X (thread: m-quad t % 4 of column group t / 4,
// t = tid % 256).  v_mfma_f32_32x32x16_bf16, 2x4 accumulators of 32x32 per wave (64 n x
// 128 k).  Measured (round 3) against the 32-row one-buffer form of wgrad_x6_kernel<4, 4>:
// 767-772 vs 790-794 us per 2-pair C2-shape call on random data, 641-644 vs 666-676 with
// L2-resident operands (the kernel is not HBM-bound); 16x16x32 MFMAs (higher clock, more
// cycles) and a register-held split of the next 32-row chunk measured equal to the old kernel.
#ifndef CN_WGRAD_DMA_NT
#define CN_WGRAD_DMA_NT 1  // wgrad_b16d_kernel's image rows loaded non-temporally (profiles/r6_ab.txt r6x)
#endif
#ifndef CN_WGRAD_NT
#define CN_WGRAD_NT 1  // wgrad_x6r_kernel's raw rows loaded non-temporally (profiles/r6_ab.txt r6w)
#endif
#ifndef CN_WGRAD_TIED_LOADS
#define CN_WGRAD_TIED_LOADS 0  // 1: measured slower (profiles/r6_ab.txt r6i)
#endif
template <int NRAW>
__global__ void __launch_bounds__(512, 2) wgrad_x6r_kernel(WgradBatch batch) {
    constexpr int BNo = 256, MC = 16, PL = 8, LSB = 3 * PL + 4;  // 28 dwords per LDS row
    constexpr int IMG = 2 * BNo * LSB;                            // one buffer: Y rows then X rows
    __shared__ __attribute__((aligned(16))) float smem[2 * IMG];

    // the job of this workgroup (scalar lookup)
    int ji = 0, b = (int)blockIdx.x;
    while (ji + 1 < batch.njobs && b >= batch.blocks[ji]) b -= batch.blocks[ji++];
    const WgradArgs& p = batch.job[ji];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware (single job): the T output tiles of one M-slice (K or N > 256) are 8 blocks apart.
    // A batch's grid is dense (nslices x T blocks per job, no padding to whole groups of 8): the
    // dispatcher deals block ids round-robin over the 8 XCDs, so padding blocks at fixed local
    // ids would leave some XCDs more working workgroups than CUs (a second round of slices)
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int tile = batch.njobs > 1 ? b % T : (b >> 3) % T;
    const int slice = batch.njobs > 1 ? b / T : (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;
    const int n0 = (tile / p.n_tiles_k) * BNo;
    const int k0 = (tile % p.n_tiles_k) * BNo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = k0 == 0 && p.bpart != nullptr;

    const bool sx = wave >= 4;  // wave-uniform: this wave stages X
    const int t = tid & 255, mq = t & 3, cg = t >> 2;
    floatx4 raw[NRAW][4];
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    auto gload = [&](int c, floatx4 (&r4)[4]) {
        const bool valid = c < total;
        const int cc = valid ? c : 0;
        const int pair = cc >= nch;
        const int mrow = mbeg + (cc - pair * nch) * MC;
        const float* src = sx ? (pair ? p.X1 : p.X0) : (pair ? p.Y1 : p.Y0);
        const int ld = sx ? (pair ? p.ldx1 : p.ldx0) : (pair ? p.ldy1 : p.ldy0);
        const int nrows = valid ? min(MC, mend - mrow) : 0;
        const int col0 = sx ? k0 : n0;
        const rsrc_t v = make_view(src + (int64_t)mrow * ld + col0, (nrows * ld - col0) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#if CN_WGRAD_TIED_LOADS
            // the load writes the set's own registers ("+v": the old value's), so the two register sets keep
            // their places across the loop's back edge -- compiled loads got fresh destinations there, and the
            // copies back (16 v_mov per two stages) waited for the loads one stage early (vmcnt(0) at the
            // back edge).  The asm loads are not counted by the compiler: wait_set() waits for them.
            const int off = ((mq * 4 + r) * ld + cg * 4) * 4;
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "+v"(r4[r]) : "v"(off), "s"(v));
#else
            r4[r] = CN_WGRAD_NT ? eload4(v, ((mq * 4 + r) * ld + cg * 4) * 4, 0) : bload4(v, ((mq * 4 + r) * ld + cg * 4) * 4, 0);
#endif
        }
    };
    // (CN_WGRAD_TIED_LOADS) a set loaded a stage ago has landed: only the 4 loads issued since may fly
    auto wait_set = [&](floatx4 (&r4)[4]) {
#if CN_WGRAD_TIED_LOADS
        asm volatile("s_waitcnt vmcnt(4)" : "+v"(r4[0]), "+v"(r4[1]), "+v"(r4[2]), "+v"(r4[3]));
#endif
    };
    // split column e of the 4 x 4 block of a register set into the stage image of buffer `buf`
    // (WB: the bias sums are taken at all -- only the Y waves of a job's first output tile; the other waves'
    // stage loop carries no bias adds)
    auto split_col = [&](auto wb_tag, const floatx4 (&r4)[4], int e, int buf, bool bias) {
        constexpr bool WB = decltype(wb_tag)::value;
        float* img = smem + buf * IMG + (sx ? BNo * LSB : 0) + mq * 2;
        const floatx4 col = {r4[0][e], r4[1][e], r4[2][e], r4[3][e]};
        if constexpr (WB) {
            // (scalar adds: a packed pair beside the MFMAs costs more issue cycles than two scalar ones)
            const float s = add_f32(add_f32(col[0], col[1]), add_f32(col[2], col[3]));
            bsum[e] = add_f32(bsum[e], bias ? s : 0.0f);
        }
        bf16x4 t0, t1, t2;
        split3(col, t0, t1, t2);
        float* y = img + (cg * 4 + e) * LSB;
        *reinterpret_cast<bf16x4*>(y) = t0;
        *reinterpret_cast<bf16x4*>(y + PL) = t1;
        *reinterpret_cast<bf16x4*>(y + 2 * PL) = t2;
    };
    auto splitw = [&](const floatx4 (&r4)[4], int buf, bool bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) split_col(std::true_type{}, r4, e, buf, bias);
    };

    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const int frow = lane & 31, fh = lane >> 5;
    constexpr int TA[6] = {0, 1, 0, 2, 1, 0};
    constexpr int TB[6] = {0, 0, 1, 0, 1, 2};
    // one stage from buffer `buf`, in four segments pinned by sched_barrier: segment j reads
    // column block j+1's B fragments, issues block j's 12 MFMAs and `side(j)` (split column j
    // of the next stage and its LDS writes), which the scheduler interleaves with the MFMAs
    auto compute = [&](int buf, auto side) {
        const float* ya = smem + buf * IMG + (wm * 64 + frow) * LSB + 4 * fh;
        const float* xa = smem + buf * IMG + BNo * LSB + (wn * 128 + frow) * LSB + 4 * fh;
        bf16x8 af[3][2], bj[2][3];
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
#pragma unroll
            for (int i = 0; i < 2; ++i) af[tt][i] = *reinterpret_cast<const bf16x8*>(ya + i * 32 * LSB + tt * PL);
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) bj[0][tt] = *reinterpret_cast<const bf16x8*>(xa + tt * PL);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j + 1 < 4) {
#pragma unroll
                for (int tt = 0; tt < 3; ++tt)
                    bj[(j + 1) & 1][tt] = *reinterpret_cast<const bf16x8*>(xa + (j + 1) * 32 * LSB + tt * PL);
            }
#pragma unroll
            for (int u = 0; u < 6; ++u)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[TA[u]][i], bj[j & 1][TB[u]], acc[i][j], 0, 0, 0);
            side(j);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // the bias sums take stage c's Y rows of pair 0 (Y threads only); bitwise, not &&, so
    // the loop body stays one basic block
    const bool ybias = do_bias & !sx;
    auto bias_of = [&](int c) { return ybias & (c < nch); };
    static_assert(!CN_WGRAD_TIED_LOADS || NRAW == 2, "wait_set counts one other set of 4 loads");
#pragma unroll
    for (int s = 0; s < NRAW; ++s) gload(s, raw[s]);
    wait_set(raw[0]);
    splitw(raw[0], 0, bias_of(0));
    __syncthreads();
    // stage c in set c % NRAW: the loop is unrolled NRAW-fold so the set indices are constants,
    // and runs whole NRAW-groups of stages (the stages past `total` read zeros: an empty view)
    auto stages = [&](auto wb_tag) {
        for (int c0 = 0; c0 < total; c0 += NRAW) {
#pragma unroll
            for (int k = 0; k < NRAW; ++k) {
                const int c = c0 + k;
                {
                    gload(c + NRAW, raw[k]);  // set k held stage c (split in the previous stage)
                    wait_set(raw[(k + 1) % NRAW]);
                    const bool bnext = bias_of(c + 1);
                    compute(c & 1, [&](int j) { split_col(wb_tag, raw[(k + 1) % NRAW], j, (c + 1) & 1, bnext); });
                    __syncthreads();  // stage c+1 written, stage c's buffer free
                }
            }
        }
    };
    if (ybias)  // (wave-uniform)
        stages(std::true_type{});
    else
        stages(std::false_type{});
    __syncthreads();  // LDS is reused for the bias partials

    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = k0 + wn * 128 + j * 32 + (lane & 31);
            const int rbase = n0 + wm * 64 + i * 32 + 4 * (lane >> 5);
            const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r) bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[i][j][r]);
        }
    }
    if (do_bias) {  // reduce the Y threads' column partials over the m-quads (fixed order)
        float* red = smem;  // [4][BNo]
        if (!sx) {
#pragma unroll
            for (int e = 0; e < 4; ++e) red[mq * BNo + cg * 4 + e] = bsum[e];
        }
        __syncthreads();
        if (tid < BNo) {
            const float tot = ((red[tid] + red[BNo + tid]) + red[2 * BNo + tid]) + red[3 * BNo + tid];
            p.bpart[(int64_t)slice * p.Npad + n0 + tid] = tot;
        }
    }
}

// Whole-layer (256x256) bf16 weight gradient (config C3's bf16 MLP MFMA) on a stage ring: the
// wgrad_x6r_kernel structure with one bf16 term per operand.  The products are the bf16 roundings
// of Y and X (RNE while staging, or read as bf16 operand images: the same bits), so dW equals
// wgrad_bf16_kernel's up to the fp32 summation order.  A stage is 32 sample rows: two buffers of
// [256 Y rows | 256 X rows] x (16 dwords of 32 bf16 + 4 pad) = 2 x 40 KB (conflict-free fragment
// reads), NRAW register sets of raw rows in flight, ONE barrier per stage; every wave does 16
// v_mfma_f32_32x32x16_bf16 per stage (2x4 accumulators of 32x32: 64 n x 128 k).  This shape is
// HBM-bound (32 KB of fp32 operands per stage for 256 MFMA cycles per SIMD), so what matters is
// the bytes in flight and reading each operand once: waves 0-3 stage Y, waves 4-7 X, each side fp32
// (m-quad t % 8 of the 4-column groups t / 8 and t / 8 + 32) or a bf16 image (m-quad t % 8 of the
// 8-column group t / 8), decided per job and side (WgradArgs::yb / xb: wave-uniform branches).
template <int NRAW>
__global__ void __launch_bounds__(512, 2) wgrad_b16r_kernel(WgradBatch batch) {
    constexpr int BNo = 256, MC = 32, PL = MC / 2, LSB = PL + 4;  // 20 dwords per LDS row
    constexpr int IMG = 2 * BNo * LSB;                              // one buffer: Y rows then X rows
    __shared__ __attribute__((aligned(16))) float smem[2 * IMG];

    int ji = 0, b = (int)blockIdx.x;
    while (ji + 1 < batch.njobs && b >= batch.blocks[ji]) b -= batch.blocks[ji++];
    const WgradArgs& p = batch.job[ji];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int tile = batch.njobs > 1 ? b % T : (b >> 3) % T;
    const int slice = batch.njobs > 1 ? b / T : (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;
    const int n0 = (tile / p.n_tiles_k) * BNo;
    const int k0 = (tile % p.n_tiles_k) * BNo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = k0 == 0 && p.bpart != nullptr;

    const bool sx = wave >= 4;                  // wave-uniform: this wave stages X
    const bool bfs = sx ? p.xb != 0 : p.yb != 0;  // wave-uniform: this side is a bf16 image
    const int t = tid & 255, mq = t & 7, cg = t >> 3;  // m-quad, column group (4 fp32 / 8 bf16 columns)
    floatx4 raw[NRAW][8];
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto gload = [&](int c, floatx4 (&r8)[8]) {
        const bool valid = c < total;
        const int cc = valid ? c : 0;
        const int pair = cc >= nch;
        const int mrow = mbeg + (cc - pair * nch) * MC;
        const float* src = sx ? (pair ? p.X1 : p.X0) : (pair ? p.Y1 : p.Y0);
        const int ld = sx ? (pair ? p.ldx1 : p.ldx0) : (pair ? p.ldy1 : p.ldy0);
        const int nrows = valid ? min(MC, mend - mrow) : 0;
        const int col0 = sx ? k0 : n0;
        if (bfs) {  // 4 rows x 8 bf16 columns
            const char* base = reinterpret_cast<const char*>(src) + ((int64_t)mrow * ld + col0) * 2;
            const rsrc_t v = make_view(reinterpret_cast<const float*>(base), (nrows * ld - col0) * 2);
#pragma unroll
            for (int r = 0; r < 4; ++r) r8[r] = bload4(v, ((mq * 4 + r) * ld + cg * 8) * 2, 0);
            // defined on both paths: with sets 4..7 left unwritten here the ring went to scratch
#pragma unroll
            for (int r = 4; r < 8; ++r) r8[r] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        } else {  // 4 rows x (4 columns of group cg, 4 of group cg + 32)
            const rsrc_t v = make_view(src + (int64_t)mrow * ld + col0, (nrows * ld - col0) * 4);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int r = 0; r < 4; ++r) r8[4 * h + r] = bload4(v, ((mq * 4 + r) * ld + (cg + 32 * h) * 4) * 4, 0);
        }
    };
    // the stage image of a register set: column c's 4 values of this m-quad as one bf16x4 at row c
    auto stage = [&](const floatx4 (&r8)[8], int buf, bool bias) {
        float* img = smem + buf * IMG + (sx ? BNo * LSB : 0) + mq * 2;
        if (bfs) {
            // rows r0..r3 as 4 dwords each (8 bf16): column 2d is the low halves of dword d, 2d + 1 the high
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                // values first: a bit cast of a vector-element lvalue reads the vector's first element
                const float f0 = r8[0][d], f1 = r8[1][d], f2 = r8[2][d], f3 = r8[3][d];
                const unsigned w0 = __builtin_bit_cast(unsigned, f0), w1 = __builtin_bit_cast(unsigned, f1);
                const unsigned w2 = __builtin_bit_cast(unsigned, f2), w3 = __builtin_bit_cast(unsigned, f3);
                const u32x2_t lo = {__builtin_amdgcn_perm(w1, w0, 0x05040100u), __builtin_amdgcn_perm(w3, w2, 0x05040100u)};
                const u32x2_t hi = {__builtin_amdgcn_perm(w1, w0, 0x07060302u), __builtin_amdgcn_perm(w3, w2, 0x07060302u)};
                *reinterpret_cast<u32x2_t*>(img + (cg * 8 + 2 * d) * LSB) = lo;
                *reinterpret_cast<u32x2_t*>(img + (cg * 8 + 2 * d + 1) * LSB) = hi;
                if (bias) {
                    bsum[2 * d] += (__builtin_bit_cast(float, w0 << 16) + __builtin_bit_cast(float, w1 << 16)) +
                                   (__builtin_bit_cast(float, w2 << 16) + __builtin_bit_cast(float, w3 << 16));
                    bsum[2 * d + 1] += (__builtin_bit_cast(float, w0 & 0xffff0000u) + __builtin_bit_cast(float, w1 & 0xffff0000u)) +
                                       (__builtin_bit_cast(float, w2 & 0xffff0000u) + __builtin_bit_cast(float, w3 & 0xffff0000u));
                }
            }
        } else {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const floatx4 col = {r8[4 * h][e], r8[4 * h + 1][e], r8[4 * h + 2][e], r8[4 * h + 3][e]};
                    if (bias) bsum[4 * h + e] += (col[0] + col[1]) + (col[2] + col[3]);
                    *reinterpret_cast<bf16x4*>(img + ((cg + 32 * h) * 4 + e) * LSB) = __builtin_convertvector(col, bf16x4);
                }
        }
    };

    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const int frow = lane & 31, fh = lane >> 5;
    auto compute = [&](int buf) {
        const float* ya = smem + buf * IMG + (wm * 64 + frow) * LSB + 4 * fh;
        const float* xa = smem + buf * IMG + BNo * LSB + (wn * 128 + frow) * LSB + 4 * fh;
#pragma unroll
        for (int ks = 0; ks < MC / 16; ++ks) {
            bf16x8 af[2], bf[4];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ya + i * 32 * LSB + ks * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const bf16x8*>(xa + j * 32 * LSB + ks * 8);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
    };

    const bool ybias = do_bias & !sx;
    auto bias_of = [&](int c) { return ybias & (c < nch); };
#pragma unroll
    for (int s = 0; s < NRAW; ++s) gload(s, raw[s]);
    stage(raw[0], 0, bias_of(0));
    __syncthreads();
    for (int c0 = 0; c0 < total; c0 += NRAW) {
#pragma unroll
        for (int k = 0; k < NRAW; ++k) {
            const int c = c0 + k;
            gload(c + NRAW, raw[k]);  // set k held stage c (staged in the previous stage)
            compute(c & 1);
            stage(raw[(k + 1) % NRAW], (c + 1) & 1, bias_of(c + 1));
            __syncthreads();  // stage c+1 written, stage c's buffer free
        }
    }
    __syncthreads();  // LDS is reused for the bias partials

    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = k0 + wn * 128 + j * 32 + (lane & 31);
            const int rbase = n0 + wm * 64 + i * 32 + 4 * (lane >> 5);
            const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r) bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[i][j][r]);
        }
    }
    if (do_bias) {  // reduce the Y threads' column partials over the 8 m-quads (fixed order)
        float* red = smem;  // [8][BNo]
        if (!sx) {
            if (p.yb) {
#pragma unroll
                for (int c = 0; c < 8; ++c) red[mq * BNo + cg * 8 + c] = bsum[c];
            } else {
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int e = 0; e < 4; ++e) red[mq * BNo + (cg + 32 * h) * 4 + e] = bsum[4 * h + e];
            }
        }
        __syncthreads();
        if (tid < BNo) {
            float tot = 0.0f;
#pragma unroll
            for (int q = 0; q < 8; ++q) tot += red[q * BNo + tid];
            p.bpart[(int64_t)slice * p.Npad + n0 + tid] = tot;
        }
    }
}

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));

// One MFMA operand (8 bf16 along the reduction) by two ds_read_b64_tr_b16 at rows r and r + 4 of a
// 512-byte-row image (ks: + 16 rows); the caller waits lgkmcnt before using it.
template <int OFF>
__device__ __forceinline__ bf16x8 tr_read8(uint32_t addr, int ks) {
    u32x2v lo, hi;
    if (ks == 0) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(addr), "i"(OFF) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(addr), "i"(OFF + 4 * 512) : "memory");
    } else {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(addr), "i"(OFF + 16 * 512) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(addr), "i"(OFF + 20 * 512) : "memory");
    }
    return __builtin_bit_cast(bf16x8, (u32x4){lo[0], lo[1], hi[0], hi[1]});
}

// The bf16 weight gradient with BOTH operands bf16 images (config C3's SDF and colour backward
// passes): the rows go HBM -> LDS by LDS-DMA (buffer_load ... lds, 16 bytes per lane), so the
// bytes in flight do not live in registers -- wgrad_b16r_kernel's register ring holds two 32-row
// stages at one workgroup per CU (~4.1 TB/s), this ring NS - 1 = 3 stages (96 KB per CU) -- and the
// MFMA operands come out of the row-major images by the transposed read ds_read_b64_tr_b16 (lane i
// of a 16-lane group gets column i of 4 rows).  A stage is 32 sample rows: [32][256] bf16 of Y then
// of X, 512-byte rows whose 16-byte chunks are XOR-swizzled by (row & 3) << 2 (the DMA writes LDS
// linearly; the swizzle is in the per-lane global address), so the four rows of a transposed read
// land in four different bank quarters: conflict-free.  The m order of every MFMA operand is
// wgrad_b16r_kernel's (m = 16 ks + 8 (lane >> 5) + e), so dW is bitwise equal to it; db sums the Y
// fragments of pair 0 in the registers (waves of the first column block), a fixed order.
template <int NS>
__global__ void __launch_bounds__(512, 2) wgrad_b16d_kernel(WgradBatch batch) {
    constexpr int BNo = 256, MC = 32, ROWB = 512;
    constexpr int SIDE = MC * ROWB, STAGE = 2 * SIDE;
    static_assert(NS >= 3 && MC == 32, "the ring keeps NS - 1 stages of two k-steps in flight");
    __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

    int ji = 0, b = (int)blockIdx.x;
    while (ji + 1 < batch.njobs && b >= batch.blocks[ji]) b -= batch.blocks[ji++];
    const WgradArgs& p = batch.job[ji];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int tile = batch.njobs > 1 ? b % T : (b >> 3) % T;
    const int slice = batch.njobs > 1 ? b / T : (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;  // (whole workgroup: no barrier is left waiting)
    const int n0 = (tile / p.n_tiles_k) * BNo;
    const int k0 = (tile % p.n_tiles_k) * BNo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = k0 == 0 && p.bpart != nullptr;

    // LDS-DMA: waves 0-3 stage Y, 4-7 X; wave w & 3 the stage rows 8 (w & 3) .. + 7, two rows
    // (1 KB) per instruction: lane l -> row + (l >> 5), physical chunk l & 31
    const bool sx = wave >= 4;
    const int wq = wave & 3;
    const int col0 = sx ? k0 : n0;
    // the side's pair-0 / pair-1 rows of this slice from col0 (wave-uniform scalars: the DMA's buffer
    // resource must sit in SGPRs)
    auto ufirst = [](int64_t x) {
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
        return (int64_t)(((uint64_t)hi << 32) | lo);
    };
    const int ld0 = sx ? p.ldx0 : p.ldy0, ld1 = sx ? p.ldx1 : p.ldy1;
    const int64_t src0 = ufirst(reinterpret_cast<int64_t>(reinterpret_cast<const bf16_t*>(sx ? p.X0 : p.Y0) +
                                                          (int64_t)mbeg * ld0 + col0));
    const int64_t src1 = p.npairs > 1 ? ufirst(reinterpret_cast<int64_t>(reinterpret_cast<const bf16_t*>(sx ? p.X1 : p.Y1) +
                                                                         (int64_t)mbeg * ld1 + col0))
                                      : src0;
    const int slice_rows = mend - mbeg;
    const int drow = (lane >> 5), dch = lane & 31;
    auto issue = [&](int c) {  // stage c (or zeros past the last: an empty view) into buffer c % NS
        const bool valid = c < total;
        const int pair = valid && c >= nch;
        const int r0 = valid ? (c - pair * nch) * MC : 0;
        const int ld = pair ? ld1 : ld0;
        // a view per chunk, based at its first row: rows past the slice's end read as zero, and no
        // byte count or offset spans the slice (int32-safe at any rows_per_slice)
        const int nrow = valid ? min(MC, slice_rows - r0) : 0;
        const int bytes = __builtin_amdgcn_readfirstlane(nrow > 0 ? (nrow * ld - col0) * 2 : 0);
        const int64_t base = (pair ? src1 : src0) + (int64_t)r0 * ld * 2;
        const rsrc_t v = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, bytes, 0x00020000);
        char* dst = smem + (c % NS) * STAGE + (sx ? SIDE : 0) + wq * 8 * ROWB;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = wq * 8 + 2 * j + drow;
            const int ch = dch ^ ((row & 3) << 2);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(v, (lds_void*)(dst + j * 1024), 16, row * ld * 2 + ch * 16,
                                                     0, 0, CN_WGRAD_DMA_NT ? 2 : 0);
        }
    };

    // transposed-read addresses: lane 4q + p of its 16-lane group g supplies row (q) of the group's
    // block, columns 4p .. 4p + 3 of its 16 (g & 1: the second 16 columns; g >> 1: rows + 8).  The
    // reads are inline asm: the compiler would otherwise drain every LDS-DMA in flight (vmcnt(0))
    // before each of them (it cannot tell the ring's buffers apart), so their lgkmcnt waits are
    // explicit too.  Per lane six addresses (Y: i = 0, 1; X: j = 0..3) within a stage; rows + 4
    // (the second half of the 8) and + 16 (ks = 1) keep row & 3, hence the swizzle: immediates.
    const int g = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
    auto tr_off = [&](int row, int col) {  // byte offset of (row, col) in a swizzled side image
        return row * ROWB + (((col >> 3) ^ ((row & 3) << 2)) << 4) + (col & 7) * 2;
    };
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
    uint32_t ya[2], xa[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) ya[i] = lds0 + tr_off(8 * (g >> 1) + tq, wm * 64 + i * 32 + 16 * (g & 1) + 4 * tp);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        xa[j] = lds0 + SIDE + tr_off(8 * (g >> 1) + tq, wn * 128 + j * 32 + 16 * (g & 1) + 4 * tp);
    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const bool bias_wave = do_bias && wn == 0;  // wave-uniform
    float bs[2] = {0.0f, 0.0f};
    auto compute = [&](int buf, bool bias) {
        const uint32_t sb = buf * STAGE;
        // both k-steps' fragments requested up front: the second's reads land under the first's MFMAs
        bf16x8 af[2][2], bf[2][4];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int i = 0; i < 2; ++i) af[ks][i] = tr_read8<0>(ya[i] + sb, ks);
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[ks][j] = tr_read8<0>(xa[j] + sb, ks);
        }
        asm volatile("s_waitcnt lgkmcnt(12)"  // (LDS reads retire in order: the first k-step's 12)
                     : "+v"(af[0][0]), "+v"(af[0][1]), "+v"(bf[0][0]), "+v"(bf[0][1]), "+v"(bf[0][2]), "+v"(bf[0][3]));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bf[0][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // the first k-step's MFMAs issue before the second's wait
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(af[1][0]), "+v"(af[1][1]), "+v"(bf[1][0]), "+v"(bf[1][1]), "+v"(bf[1][2]), "+v"(bf[1][3]));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bf[1][j], acc[i][j], 0, 0, 0);
        if (bias) {  // this lane's column of Y over its 16 rows of the stage, in m order
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float sm = 0.0f;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const u32x4 w = __builtin_bit_cast(u32x4, af[ks][i]);
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        sm += __builtin_bit_cast(float, w[e] << 16) + __builtin_bit_cast(float, w[e] & 0xffff0000u);
                }
                bs[i] += sm;
            }
        }
    };

#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(s);
    for (int c = 0; c < total; ++c) {
        wait_vmcnt<4 * (NS - 2)>();  // this wave's DMAs of stage c landed (NS - 2 later stages may fly)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's stage c landed; every wave is done with stage c - 1
        asm volatile("" ::: "memory");
        issue(c + NS - 1);  // into the buffer stage c - 1 used
        compute(c % NS, bias_wave && c < nch);
    }
    wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    __syncthreads();  // LDS is reused for the bias partials

    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = k0 + wn * 128 + j * 32 + (lane & 31);
            const int rbase = n0 + wm * 64 + i * 32 + 4 * (lane >> 5);
            const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r) bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[i][j][r]);
        }
    }
    if (do_bias) {  // the two row halves of each column (lanes l, l + 32), fixed order
        float* red = reinterpret_cast<float*>(smem);  // [2][BNo]
        if (bias_wave) {
#pragma unroll
            for (int i = 0; i < 2; ++i) red[(lane >> 5) * BNo + wm * 64 + i * 32 + (lane & 31)] = bs[i];
        }
        __syncthreads();
        if (tid < BNo) p.bpart[(int64_t)slice * p.Npad + n0 + tid] = red[tid] + red[BNo + tid];
    }
}

// 256 x 64 weight gradient (the K = 64 first layers: the SDF's dW0 = Z_0ᵀ U0 + S_0ᵀ U̇_0 and the colour
// network's extras columns, neus_fields.py:268-272, 364-366) on the stage ring of wgrad_x6r_kernel:
// 16 sample rows per stage, two split-image buffers (2 x 35 KB: 256 Y rows + 64 X rows of 28 dwords),
// NRAW register sets of raw rows in flight, one barrier per stage.  These shapes move ~6 bytes per
// bf16x6 FLOP-pair more than the 256-wide layers (HBM-bound), so the ring keeps NRAW stages of loads in
// flight and every wave does MFMA work: wave w owns output rows 32w .. 32w+31 (1 x 2 accumulators of
// 32 x 32).  Waves 0-3 stage Y (m-quad t % 4 of column group t / 4), wave 4 stages X.
template <int NRAW>
__global__ void __launch_bounds__(512, 4) wgrad_x6n_kernel(WgradArgs p) {  // 2 per CU: <= 128 VGPRs
    constexpr int BNo = 256, BKo = 64, MC = 16, PL = 8, LSB = 3 * PL + 4;
    constexpr int IMG = (BNo + BKo) * LSB;
    __shared__ __attribute__((aligned(16))) float smem[2 * IMG];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.n_tiles_n * p.n_tiles_k;
    const int b = blockIdx.x;
    const int tile = (b >> 3) % T;
    const int slice = (b & 7) + 8 * ((b >> 3) / T);
    if (slice >= p.nslices) return;
    const int n0 = (tile / p.n_tiles_k) * BNo;
    const int k0 = (tile % p.n_tiles_k) * BKo;
    const int mbeg = slice * p.rows_per_slice;
    const int mend = min(p.M, mbeg + p.rows_per_slice);
    const int nch = mend > mbeg ? cdiv(mend - mbeg, MC) : 0;
    const int total = nch * p.npairs;
    const bool do_bias = k0 == 0 && p.bpart != nullptr;

    const bool sy = wave < 4;    // wave-uniform staging roles: Y (waves 0-3), X (wave 4), none (5-7)
    const bool sxw = wave == 4;
    const bool stager = sy || sxw;
    const int t = tid & 255, mq = t & 3, cg = t >> 2;
    floatx4 raw[NRAW][4];
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    auto gload = [&](int c, floatx4 (&r4)[4]) {
        if (!stager) return;  // waves 5-7 stage nothing (their raw sets are never read)
        const bool valid = c < total;
        const int cc = c < total ? c : 0;
        const int pair = cc >= nch;
        const int mrow = mbeg + (cc - pair * nch) * MC;
        const float* src = sy ? (pair ? p.Y1 : p.Y0) : (pair ? p.X1 : p.X0);
        const int ld = sy ? (pair ? p.ldy1 : p.ldy0) : (pair ? p.ldx1 : p.ldx0);
        const int nrows = valid ? min(MC, mend - mrow) : 0;
        const int col0 = sy ? n0 : k0;
        const rsrc_t v = make_view(src + (int64_t)mrow * ld + col0, (nrows * ld - col0) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) r4[r] = bload4(v, ((mq * 4 + r) * ld + cg * 4) * 4, 0);
    };
    auto split_col = [&](const floatx4 (&r4)[4], int e, int buf, bool bias) {
        if (!stager) return;
        float* img = smem + buf * IMG + (sy ? 0 : BNo * LSB) + mq * 2;
        const floatx4 col = {r4[0][e], r4[1][e], r4[2][e], r4[3][e]};
        const float sm = add_f32(add_f32(col[0], col[1]), add_f32(col[2], col[3]));
        bsum[e] = add_f32(bsum[e], bias ? sm : 0.0f);
        bf16x4 t0, t1, t2;
        split3(col, t0, t1, t2);
        float* y = img + (cg * 4 + e) * LSB;
        *reinterpret_cast<bf16x4*>(y) = t0;
        *reinterpret_cast<bf16x4*>(y + PL) = t1;
        *reinterpret_cast<bf16x4*>(y + 2 * PL) = t2;
    };

    floatx16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
    const int frow = lane & 31, fh = lane >> 5;
    constexpr int TA[6] = {0, 1, 0, 2, 1, 0};
    constexpr int TB[6] = {0, 0, 1, 0, 1, 2};
    // one stage in two segments: segment j issues k block j's 6 MFMAs beside split columns 2j, 2j+1
    auto compute = [&](int buf, auto side) {
        const float* ya = smem + buf * IMG + (wave * 32 + frow) * LSB + 4 * fh;
        const float* xa = smem + buf * IMG + BNo * LSB + frow * LSB + 4 * fh;
        bf16x8 af[3], bj[3];
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) af[tt] = *reinterpret_cast<const bf16x8*>(ya + tt * PL);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int tt = 0; tt < 3; ++tt) bj[tt] = *reinterpret_cast<const bf16x8*>(xa + j * 32 * LSB + tt * PL);
#pragma unroll
            for (int u = 0; u < 6; ++u)
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[TA[u]], bj[TB[u]], acc[j], 0, 0, 0);
            side(2 * j);
            side(2 * j + 1);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    const bool ybias = do_bias & sy;
    auto bias_of = [&](int c) { return ybias & (c < nch); };
#pragma unroll
    for (int st = 0; st < NRAW; ++st) gload(st, raw[st]);
#pragma unroll
    for (int e = 0; e < 4; ++e) split_col(raw[0], e, 0, bias_of(0));
    __syncthreads();
    for (int c0 = 0; c0 < total; c0 += NRAW) {
#pragma unroll
        for (int k = 0; k < NRAW; ++k) {
            const int c = c0 + k;
            gload(c + NRAW, raw[k]);  // set k held stage c (split in the previous stage)
            const bool bnext = bias_of(c + 1);
            compute(c & 1, [&](int e) { split_col(raw[(k + 1) % NRAW], e, (c + 1) & 1, bnext); });
            __syncthreads();  // stage c+1 written, stage c's buffer free
        }
    }
    __syncthreads();  // LDS is reused for the bias partials

    const rsrc_t vP = make_view(p.part + (int64_t)slice * p.Npad * p.Kpad, p.Npad * p.Kpad * 4);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = k0 + j * 32 + (lane & 31);
        const int rbase = n0 + wave * 32 + 4 * (lane >> 5);
        const int vo = (rbase * p.Kpad + col) * 4;
#pragma unroll
        for (int r = 0; r < 16; ++r) bstore1(vP, vo, ((r & 3) + 8 * (r >> 2)) * p.Kpad * 4, acc[j][r]);
    }
    if (do_bias) {  // reduce the Y threads' column partials over the m-quads (fixed order)
        float* red = smem;  // [4][BNo]
        if (sy) {
#pragma unroll
            for (int e = 0; e < 4; ++e) red[mq * BNo + cg * 4 + e] = bsum[e];
        }
        __syncthreads();
        if (tid < BNo) {
            const float tot = ((red[tid] + red[BNo + tid]) + red[2 * BNo + tid]) + red[3 * BNo + tid];
            p.bpart[(int64_t)slice * p.Npad + n0 + tid] = tot;
        }
    }
}

// Sum of nslab fp32 slabs: out[r*ldo + c] (+)= (sum_s part[s*stride + r*ldp + c]) / div
// for r < rows, c < cols.  A workgroup owns 64 float4 column groups x 4 slab
// groups; each thread sums its slab group in double with 4 loads in flight, the 4
// groups combine through LDS in a fixed order (bitwise reproducible).
// 256 threads = kSlabGroups slab groups x (256 / kSlabGroups) float4 column groups: slab
// group sg sums slabs sg, sg + SG, ... in double, the groups meet in a fixed order in LDS.
// (16 x 16: a 256-slab weight gradient is 16 loads per thread, 4x the blocks of a 4 x 64 split.)
constexpr int kSlabGroups = 16;
constexpr int kSlabCG = 256 / kSlabGroups;  // float4 column groups per workgroup

SlabJob slab_job(const float* part, int nslab, int64_t stride, int rows, int cols, int64_t ldp, float* out,
                 int64_t ldo, float div, int accumulate) {
    const int64_t groups = (int64_t)rows * cdiv(cols, 4);
    return SlabJob{part, out, stride, ldp, ldo, nslab, rows, cols, accumulate,
                   (int)((groups + kSlabCG - 1) / kSlabCG), div};
}

// Several reductions in one launch (a weight gradient's dW and db, or every job of a batched
// weight gradient): job i takes the next j[i].blocks workgroups -- one launch and one tail.
__global__ void __launch_bounds__(256) slab_reduce_kernel(SlabBatch jobs) {
    constexpr int SG = kSlabGroups, CG = kSlabCG;
    __shared__ double red[SG][CG][4];
    int ji = 0, blk = (int)blockIdx.x;  // workgroup-uniform job lookup (scalar)
    while (ji + 1 < jobs.n && blk >= jobs.j[ji].blocks) blk -= jobs.j[ji++].blocks;
    const SlabJob& j = jobs.j[ji];
    const int c4n = cdiv(j.cols, 4);
    const int t = threadIdx.x % CG;
    const int sg = threadIdx.x / CG;
    const int64_t g = (int64_t)blk * CG + t;  // float4 group over rows x c4n
    const bool valid = g < (int64_t)j.rows * c4n;
    const int r = valid ? (int)(g / c4n) : 0;
    const int c = valid ? (int)(g % c4n) * 4 : 0;
    const bool vec = valid && (c + 3 < j.cols) && (j.ldp % 4 == 0) && (j.stride % 4 == 0);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    if (valid) {
        const float* base = j.part + (int64_t)r * j.ldp + c;
        int sl = sg;
        for (; sl + 3 * SG < j.nslab; sl += 4 * SG) {
            floatx4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float* q = base + (int64_t)(sl + SG * u) * j.stride;
                if (vec) {
                    v[u] = *reinterpret_cast<const floatx4*>(q);
                } else {
                    for (int e = 0; e < 4; ++e) v[u][e] = (c + e < j.cols) ? q[e] : 0.0f;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) a[e] += (double)v[u][e];
        }
        for (; sl < j.nslab; sl += SG) {
            const float* q = base + (int64_t)sl * j.stride;
            for (int e = 0; e < 4; ++e) a[e] += (c + e < j.cols) ? (double)q[e] : 0.0;
        }
    }
    for (int e = 0; e < 4; ++e) red[sg][t][e] = a[e];
    __syncthreads();
    if (sg == 0 && valid) {
        for (int e = 0; e < 4 && c + e < j.cols; ++e) {
            double tot = red[0][t][e];
            for (int q = 1; q < SG; ++q) tot += red[q][t][e];
            float v = (float)tot;
            if (j.div != 1.0f) v = v / j.div;
            float* o = j.out + (int64_t)r * j.ldo + c + e;
            if (j.accumulate) v += *o;
            *o = v;
        }
    }
}

int launch_slab_batch(const SlabJob* jobs, int n, hipStream_t s) {
    CN_REQUIRE(n >= 0 && n <= kSlabMax, CN_ERR_ARG, "slab_reduce: %d jobs (at most %d)", n, kSlabMax);
    SlabBatch b{};
    int blocks = 0;
    for (int i = 0; i < n; ++i) {
        if (jobs[i].blocks == 0) continue;  // empty job (e.g. no db)
        b.j[b.n++] = jobs[i];
        blocks += jobs[i].blocks;
    }
    if (blocks == 0) return CN_OK;
    slab_reduce_kernel<<<blocks, 256, 0, s>>>(b);
    return check_launch("slab_reduce");
}

int launch_slab_jobs(const SlabJob& j0, const SlabJob& j1, hipStream_t s) {
    const SlabJob jobs[2] = {j0, j1};
    return launch_slab_batch(jobs, 2, s);
}

int launch_slab_reduce(const float* part, int nslab, int64_t stride, int rows, int cols, int64_t ldp, float* out,
                       int64_t ldo, float div, int accumulate, hipStream_t s) {
    SlabJob none{};
    return launch_slab_jobs(slab_job(part, nslab, stride, rows, cols, ldp, out, ldo, div, accumulate), none, s);
}

// ---------------------------------------------------------------------------
// tile 0: 128x128 output tiles, 1: 128x64, 2 (bf16x6, operand rows at least 256-padded):
// 256x256 tiles of 512-thread workgroups on the stage ring, one per CU, 3 (bf16x6, K <= 64, Y
// rows 256-padded): 256x64 tiles on the narrow stage ring.  Padding columns of Y / X only feed
// output rows / columns past n_out / k_out, which the slab reduction never reads.
// Returns the wide mode: 0 none, 1 = 256x256, 2 = 256x64.
// bf16 (CN_MFMA_BF16): 256x256 tiles on the bf16 stage ring (wgrad_b16r_kernel) when the operand
// rows are 256-padded, else the 128x128 / 128x64 tiles of wgrad_bf16_kernel (fp32 operands).
static int wgrad_wide(const cn_wgrad_desc* d) {
    const int64_t np = (int64_t)cdiv(d->N, 256) * 256, kp = (int64_t)cdiv(d->K, 256) * 256;
    const bool x6 = d->mfma_dtype == CN_MFMA_F32_BF16X6, bf = d->mfma_dtype == CN_MFMA_BF16;
    if (!(x6 || bf) || d->ldy0 < np || (d->npairs == 2 && d->ldy1 < np)) return 0;
    if (d->ldx0 >= kp && (d->npairs == 1 || d->ldx1 >= kp)) return 1;
    return x6 && d->K <= 64 ? 2 : 0;
}

// budget: workgroups this weight gradient may use (< 0: the default target; cn_wgrad_batch hands
// each job its share of one launch)
static void wgrad_geometry(int M, int N, int K, int wide, int* tile, int* Npad, int* Kpad, int* nslices,
                           int* rows_per_slice, int budget = -1) {
    const int t = wide == 1 ? 2 : wide == 2 ? 3 : (K % 128 == 0) ? 0 : 1;
    const int BNo = t >= 2 ? 256 : 128, BKo = t == 2 ? 256 : t == 0 ? 128 : 64;
    *tile = t;
    *Npad = cdiv(N, BNo) * BNo;
    *Kpad = cdiv(K, BKo) * BKo;
    const int tiles = (*Npad / BNo) * (*Kpad / BKo);
    constexpr int kTarget = 512;  // workgroups per cn_wgrad (two per CU; the 256x256 tiles one per CU)
    const int target = budget >= 0 ? budget : (t == 2 ? kTarget / 2 : kTarget);
    int ns = std::max(1, target / tiles);
    ns = std::min(ns, std::max(1, cdiv(M, 512)));
    int rps = cdiv(cdiv(M, ns), 64) * 64;  // whole 32-row (fp32) / 64-row (bf16) chunks
    ns = std::max(1, cdiv(M, rps));
    *nslices = ns;
    *rows_per_slice = rps;
}

// The CU count of the current device, cached per device (the batch's slice layout -- and so the
// fixed summation order of dW -- follows it).
static int wgrad_device_cus() {
    static thread_local int cached_dev = -1, cached_cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev != cached_dev) {
        int v = 0;
        cached_cus = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
        cached_dev = dev;
    }
    return cached_cus;
}

}  // namespace cn

using namespace cn;

// The split-M kernel cn_wgrad launches for a descriptor (its fixed-order slab reduction,
// cn::slab_reduce_kernel, follows it), decided by the same geometry as the launch.
extern "C" int cn_wgrad_kernel_name(const cn_wgrad_desc* d, char* buf, int32_t len) {
    CN_REQUIRE(d && buf && len > 0, CN_ERR_ARG, "cn_wgrad_kernel_name: null desc / buffer");
    int tile, Npad, Kpad, ns, rps;
    wgrad_geometry(std::max(d->M, 1), d->N, d->K, wgrad_wide(d), &tile, &Npad, &Kpad, &ns, &rps);
    const char* k = "";
    if (d->mfma_dtype == CN_MFMA_F32_BF16X6)
        k = tile == 2 ? "wgrad_x6r_kernel<2>" : tile == 3 ? "wgrad_x6n_kernel<3>" : tile == 0 ? "wgrad_x6_kernel<2, 2>"
                                                                                       : "wgrad_x6_kernel<2, 1>";
    else if (d->mfma_dtype == CN_MFMA_BF16)
        k = tile == 2 ? (d->y_bf16 && d->x_bf16 ? "wgrad_b16d_kernel<4>" : "wgrad_b16r_kernel<2>")
                      : tile == 0 ? "wgrad_bf16_kernel<2, 2, 2, 2>" : "wgrad_bf16_kernel<2, 2, 2, 1>";
    else
        k = tile == 0 ? "wgrad_kernel<2, 2, 2, 2>" : "wgrad_kernel<2, 2, 2, 1>";
    const bool ring = (d->mfma_dtype == CN_MFMA_F32_BF16X6 || d->mfma_dtype == CN_MFMA_BF16) && tile == 2;
    const int n = snprintf(buf, (size_t)len, "void cn::%s(cn::%s)", k, ring ? "WgradBatch" : "WgradArgs");
    CN_REQUIRE(n < len, CN_ERR_SHAPE, "cn_wgrad_kernel_name: buffer of %d bytes too small (%d)", len, n + 1);
    return n;
}

extern "C" size_t cn_wgrad_workspace_bytes(int32_t M, int32_t N, int32_t K) {
    size_t need = 0;  // the largest of the tilings (the call's mfma_dtype and leading dimensions pick one)
    for (int w = 0; w < 3; ++w) {
        int tile, Npad, Kpad, ns, rps;
        wgrad_geometry(std::max(M, 1), N, K, w, &tile, &Npad, &Kpad, &ns, &rps);
        need = std::max(need, sizeof(float) * ((size_t)ns * Npad * Kpad + (size_t)ns * Npad));
    }
    return need;
}

// The workspace one weight gradient needs with a workgroup budget (its slabs of dW and db).
static size_t wgrad_need(const cn_wgrad_desc* d, int budget) {
    int tile, Npad, Kpad, ns, rps;
    wgrad_geometry(std::max(d->M, 1), d->N, d->K, wgrad_wide(d), &tile, &Npad, &Kpad, &ns, &rps, budget);
    return sizeof(float) * ((size_t)ns * Npad * Kpad + (size_t)ns * Npad);
}

// Checks a descriptor and lays out its launch: kernel arguments, the tile class, the grid and
// the slab reductions of dW and db.  budget as in wgrad_geometry.
static int wgrad_plan(const cn_wgrad_desc* d, int budget, WgradArgs* a, int* tile_out, int* grid_out, SlabJob* jw,
                      SlabJob* jb) {
    CN_REQUIRE(d, CN_ERR_ARG, "cn_wgrad: null desc");
    CN_REQUIRE(d->Y0 && d->X0 && d->dW && d->workspace, CN_ERR_ARG, "cn_wgrad: Y0, X0, dW, workspace required");
    CN_REQUIRE(d->npairs == 1 || (d->npairs == 2 && d->Y1 && d->X1), CN_ERR_ARG, "cn_wgrad: bad npairs");
    CN_REQUIRE(d->M >= 0 && d->N > 0 && d->K > 0 && d->K % 64 == 0, CN_ERR_SHAPE,
               "cn_wgrad: bad shape M=%d N=%d K=%d (K must be a multiple of 64)", d->M, d->N, d->K);
    CN_REQUIRE(d->mfma_dtype == CN_MFMA_F32 || d->mfma_dtype == CN_MFMA_BF16 || d->mfma_dtype == CN_MFMA_F32_BF16X6,
               CN_ERR_ARG, "cn_wgrad: bad mfma_dtype %d", d->mfma_dtype);
    int tile, Npad, Kpad, ns, rps;
    wgrad_geometry(std::max(d->M, 1), d->N, d->K, wgrad_wide(d), &tile, &Npad, &Kpad, &ns, &rps, budget);
    if (d->y_bf16 || d->x_bf16)  // bf16 operand images (ABI v10): the bf16 stage ring only
        CN_REQUIRE(d->mfma_dtype == CN_MFMA_BF16 && tile == 2 && (!d->y_bf16 || (d->ldy0 % 8 == 0 && d->ldy1 % 8 == 0)) &&
                       (!d->x_bf16 || (d->ldx0 % 8 == 0 && d->ldx1 % 8 == 0)),
                   CN_ERR_UNSUPPORTED, "cn_wgrad: bf16 operand images need CN_MFMA_BF16, 256-padded operand rows and "
                   "leading dimensions % 8 == 0");
    CN_REQUIRE(d->n_out <= Npad && d->k_out <= Kpad && d->n_out > 0 && d->k_out > 0, CN_ERR_SHAPE, "cn_wgrad: bad n_out/k_out");
    CN_REQUIRE(d->ldy0 >= Npad && d->ldx0 >= Kpad && d->ldy0 % 4 == 0 && d->ldx0 % 4 == 0 && al16(d->Y0) && al16(d->X0),
               CN_ERR_ALIGN, "cn_wgrad: Y0/X0 must be 16B aligned with ld >= padded tile (%d, %d)", Npad, Kpad);
    if (d->npairs == 2)
        CN_REQUIRE(d->ldy1 >= Npad && d->ldx1 >= Kpad && d->ldy1 % 4 == 0 && d->ldx1 % 4 == 0 && al16(d->Y1) && al16(d->X1),
                   CN_ERR_ALIGN, "cn_wgrad: Y1/X1 alignment");
    CN_REQUIRE(d->ldy0 < (1 << 20) && d->ldx0 < (1 << 20) && d->ldy1 < (1 << 20) && d->ldx1 < (1 << 20), CN_ERR_SHAPE,
               "cn_wgrad: leading dimensions must be < 2^20");
    const size_t need = wgrad_need(d, budget);  // <= cn_wgrad_workspace_bytes (ns <= the default's)
    CN_REQUIRE((size_t)d->workspace_bytes >= need, CN_ERR_SHAPE, "cn_wgrad: workspace %lld < %zu", (long long)d->workspace_bytes, need);
    a->Y0 = static_cast<const float*>(d->Y0); a->X0 = static_cast<const float*>(d->X0);
    a->Y1 = static_cast<const float*>(d->Y1); a->X1 = static_cast<const float*>(d->X1);
    a->part = d->workspace;
    a->bpart = d->db ? d->workspace + (size_t)ns * Npad * Kpad : nullptr;
    a->ldy0 = (int)d->ldy0; a->ldx0 = (int)d->ldx0; a->ldy1 = (int)d->ldy1; a->ldx1 = (int)d->ldx1;
    a->M = d->M; a->Npad = Npad; a->Kpad = Kpad; a->npairs = d->npairs; a->rows_per_slice = rps;
    const int BNo = tile >= 2 ? 256 : 128, BKo = tile == 2 ? 256 : tile == 0 ? 128 : 64;
    a->n_tiles_k = Kpad / BKo;
    a->n_tiles_n = Npad / BNo;
    a->nslices = ns;
    a->yb = d->y_bf16 ? 1 : 0;
    a->xb = d->x_bf16 ? 1 : 0;
    *tile_out = tile;
    *grid_out = cdiv(ns, 8) * 8 * a->n_tiles_n * a->n_tiles_k;
    // dW and db (when asked for) in one reduction launch
    *jw = slab_job(a->part, ns, (int64_t)Npad * Kpad, d->n_out, d->k_out, Kpad, d->dW, d->ld_dw, 1.0f, d->accumulate);
    *jb = d->db ? slab_job(a->bpart, ns, Npad, 1, d->n_out, Npad, d->db, d->n_out, 1.0f, d->accumulate) : SlabJob{};
    return CN_OK;
}

extern "C" int cn_wgrad(const cn_wgrad_desc* d, cn_stream_t stream) {
    WgradArgs a;
    int tile, grid;
    SlabJob js[2];
    int rc = wgrad_plan(d, -1, &a, &tile, &grid, &js[0], &js[1]);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (d->mfma_dtype == CN_MFMA_F32_BF16X6) {
        if (tile == 2) {
            WgradBatch b{};
            b.job[0] = a;
            b.blocks[0] = grid;
            b.njobs = 1;
            wgrad_x6r_kernel<2><<<grid, 512, 0, s>>>(b);
        } else if (tile == 3) {
            wgrad_x6n_kernel<3><<<grid, 512, 0, s>>>(a);
        } else if (tile == 0) {
            wgrad_x6_kernel<2, 2><<<grid, 256, 0, s>>>(a);
        } else {
            wgrad_x6_kernel<2, 1><<<grid, 256, 0, s>>>(a);
        }
    } else if (d->mfma_dtype == CN_MFMA_BF16) {
        if (tile == 2) {
            WgradBatch b{};
            b.job[0] = a;
            b.blocks[0] = grid;
            b.njobs = 1;
            if (a.yb && a.xb)
                wgrad_b16d_kernel<4><<<grid, 512, 0, s>>>(b);
            else
                wgrad_b16r_kernel<2><<<grid, 512, 0, s>>>(b);
        } else if (tile == 0)
            wgrad_bf16_kernel<2, 2, 2, 2><<<grid, 256, 0, s>>>(a);
        else
            wgrad_bf16_kernel<2, 2, 2, 1><<<grid, 256, 0, s>>>(a);
    } else if (tile == 0) {
        wgrad_kernel<2, 2, 2, 2><<<grid, 256, 0, s>>>(a);
    } else {
        wgrad_kernel<2, 2, 2, 1><<<grid, 256, 0, s>>>(a);
    }
    rc = check_launch("cn_wgrad");
    return rc ? rc : launch_slab_batch(js, 2, s);
}

// Whether cn_wgrad_batch runs a descriptor inside a shared stage-ring launch (1: bf16x6, 2: bf16,
// 3: bf16 with both operands images -- wgrad_b16d_kernel).
constexpr int kWgradKinds = 3;
static int wgrad_batchable(const cn_wgrad_desc* d) {
    if (wgrad_wide(d) != 1) return 0;
    if (d->mfma_dtype == CN_MFMA_F32_BF16X6) return 1;
    if (d->mfma_dtype == CN_MFMA_BF16) return d->y_bf16 && d->x_bf16 ? 3 : 2;
    return 0;
}

// The batch layout of cn_wgrad_batch: the stage-ring descriptors of each kind (wgrad_batchable; at
// most kWgradBatchMax each) share one launch, each with a share of the device's workgroups
// proportional to its work (rows x pairs x output tiles), so they end together; budget[i] = -1:
// descriptor i runs alone (cn_wgrad).  kind[i] as wgrad_batchable.
static void wgrad_batch_layout(const cn_wgrad_desc* descs, int n, int* kind, int* budget) {
    double total[kWgradKinds] = {};
    int cnt[kWgradKinds] = {};
    for (int i = 0; i < n; ++i) {
        const cn_wgrad_desc* d = descs + i;
        kind[i] = wgrad_batchable(d);
        budget[i] = -1;
        if (kind[i] == 0 || cnt[kind[i] - 1] == kWgradBatchMax) {
            kind[i] = 0;
            continue;
        }
        cnt[kind[i] - 1]++;
        total[kind[i] - 1] += (double)std::max(d->M, 1) * d->npairs * cdiv(d->N, 256) * cdiv(d->K, 256);
    }
    const int cus = wgrad_device_cus();
    for (int i = 0; i < n; ++i) {
        if (kind[i] == 0) continue;
        const cn_wgrad_desc* d = descs + i;
        const int tiles = cdiv(d->N, 256) * cdiv(d->K, 256);
        const double work = (double)std::max(d->M, 1) * d->npairs * tiles;
        // floor of the proportional share: the slices of all jobs never exceed one workgroup per CU
        budget[i] = std::max(tiles, (int)(cus * work / total[kind[i] - 1]) / tiles * tiles);
    }
}

// One shared launch of a stage-ring kernel (kind as wgrad_batchable) over the descriptors idx[0..nb)
// with their budgets, then one slab reduction.
static int wgrad_ring_batch(const cn_wgrad_desc* descs, const int* idx, const int* budgets, int nb, int kind,
                            hipStream_t s) {
    if (nb == 0) return CN_OK;
    WgradBatch b{};
    SlabJob js[2 * kWgradBatchMax];
    int grid = 0;
    for (int q = 0; q < nb; ++q) {
        const cn_wgrad_desc* d = descs + idx[q];
        int tile, g;
        int rc = wgrad_plan(d, budgets[idx[q]], &b.job[q], &tile, &g, &js[2 * q], &js[2 * q + 1]);
        if (rc) return rc;
        g = b.job[q].nslices * b.job[q].n_tiles_n * b.job[q].n_tiles_k;  // dense (see the kernel)
        b.blocks[q] = g;
        grid += g;
    }
    b.njobs = nb;
    if (nb == 1) b.blocks[0] = grid = cdiv(b.job[0].nslices, 8) * 8 * b.job[0].n_tiles_n * b.job[0].n_tiles_k;
    if (kind == 1)
        wgrad_x6r_kernel<2><<<grid, 512, 0, s>>>(b);
    else if (kind == 3)
        wgrad_b16d_kernel<4><<<grid, 512, 0, s>>>(b);
    else
        wgrad_b16r_kernel<2><<<grid, 512, 0, s>>>(b);
    int rc = check_launch("cn_wgrad_batch");
    return rc ? rc : launch_slab_batch(js, 2 * nb, s);
}

extern "C" size_t cn_wgrad_batch_workspace_bytes(const cn_wgrad_desc* descs, int32_t n, int64_t* offsets) {
    if (!descs || n <= 0 || n > 4 * kWgradBatchMax) return 0;
    int kind[4 * kWgradBatchMax], budget[4 * kWgradBatchMax];
    wgrad_batch_layout(descs, n, kind, budget);
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        if (offsets) offsets[i] = (int64_t)off;
        off += (wgrad_need(descs + i, budget[i]) + 255) / 256 * 256;
    }
    return off;
}

extern "C" int cn_wgrad_batch(const cn_wgrad_desc* descs, int32_t n, cn_stream_t stream) {
    CN_REQUIRE(descs && n >= 0 && n <= 4 * kWgradBatchMax, CN_ERR_ARG, "cn_wgrad_batch: null descs / n outside [0, %d]",
               4 * kWgradBatchMax);
    hipStream_t s = (hipStream_t)stream;
    int kind[4 * kWgradBatchMax], budget[4 * kWgradBatchMax];
    wgrad_batch_layout(descs, n, kind, budget);
    int idx[kWgradKinds][kWgradBatchMax], nb[kWgradKinds] = {};
    for (int i = 0; i < n; ++i) {
        if (kind[i] == 0) {
            int rc = cn_wgrad(descs + i, stream);  // another tile class (or a full batch): its own launch
            if (rc) return rc;
            continue;
        }
        idx[kind[i] - 1][nb[kind[i] - 1]++] = i;
    }
    for (int k = 1; k <= kWgradKinds; ++k) {
        int rc = wgrad_ring_batch(descs, idx[k - 1], budget, nb[k - 1], k, s);
        if (rc) return rc;
    }
    return CN_OK;
}
