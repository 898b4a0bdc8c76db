/* copenerf.h — C ABI of libcopenerf.so, the MI355X (gfx950) kernels behind the
 * cope-nerf NeuS volumetric-rendering hot path.
 *
 * The reference (HoangChuongNguyen/cope-nerf) is pure PyTorch: it has no FFI.
 * Each entry point below replaces one group of aten calls on the hot path and
 * cites the reference lines it restates (paths relative to the reference root).
 * The host side that binds these symbols is cope-nerf_amd/copenerf/_lib.py
 * (ctypes); INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *  - All pointers are device pointers (fp32 unless typed otherwise), row-major,
 *    with explicit leading dimensions in ELEMENTS.  The caller owns all memory.
 *  - `stream` is a hipStream_t (passed as void* so that this header needs no HIP
 *    headers).  Nothing here allocates, synchronises, or uses the null stream:
 *    any sequence of calls is hipGraph-capturable and re-entrant across devices
 *    (torch.nn.DataParallel runs one host thread per GPU, train.py:54).
 *  - Return 0 on success, a negative cn_status on a bad argument or a failed
 *    launch; cn_last_error() holds the message (thread-local).  Asynchronous
 *    device faults surface at the caller's next synchronisation.
 */
#ifndef COPENERF_H_
#define COPENERF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CN_ABI_VERSION 15

typedef void* cn_stream_t; /* hipStream_t */

typedef enum cn_status {
    CN_OK = 0,
    CN_ERR_ARG = -1,         /* null pointer / bad enum */
    CN_ERR_SHAPE = -2,       /* inconsistent sizes or leading dimensions */
    CN_ERR_ALIGN = -3,       /* pointer / leading dimension not 16-byte aligned */
    CN_ERR_LAUNCH = -4,      /* hipLaunchKernel failed */
    CN_ERR_UNSUPPORTED = -5  /* configuration outside what the kernels implement */
} cn_status;

int cn_abi_version(void);
const char* cn_last_error(void);

/* ------------------------------------------------------------------------ *
 * Fully-connected layers: out = epilogue((A · Bᵀ) / adiv [+ rowv ⊗ colv])
 * Replaces every nn.Linear of SDFNetwork (model/neus_fields.py:273-283) and
 * RenderingNetwork (model/neus_fields.py:364-370), the first-order backward of
 * those layers (autograd of the same lines), the ∇ₓSDF pass of
 * SDFNetwork.gradient (neus_fields.py:291-303) and its create_graph double
 * backward.  Computed with v_mfma_f32_32x32x2_f32 (exact fp32 products).
 *
 *   A   : [M][>=K] (lda), optionally a virtual concat: columns k < K1 come from
 *         A, columns k >= K1 from A2 (column k-K1).  K, K1 multiples of 32.
 *   B   : [Npad][K] (ldb), Npad = N rounded up to the tile width (128, or 64
 *         when tile == 1); rows >= N must be readable (zero-padded weights).
 *   Columns [0, N) of out0 get the epilogue value, columns [N, nzero) get 0.
 * ------------------------------------------------------------------------ */
/* sg(x) = 1 - exp(-aux_beta * x): softplus'(z) recovered from a stored softplus
 * output x = softplus_beta(z) / c (aux_beta = beta * c), since exp(beta a) = 1 +
 * exp(beta z).  The derivative is never stored (ABI v4): the backward reads the
 * activations it already keeps. */
typedef enum cn_epilogue {
    CN_EPI_STORE = 0,        /* out0 = v + bias                                      */
    CN_EPI_SOFTPLUS = 1,     /* z = v + bias; out0 = softplus_beta(z)/odiv           */
    CN_EPI_RELU = 2,         /* out0 = relu(v + bias)                                */
    CN_EPI_MUL = 3,          /* out0 = v * sg(aux0) (cols < nsplit); out_split = v (cols >= nsplit) */
    CN_EPI_TANGENT = 4,      /* out0 = v * sg(aux0) / odiv                           */
    CN_EPI_BWD_SOFTPLUS = 5, /* out0 = v*sg(aux0) + aux1*aux2*aux2_scale*(1-sg)/sg (0 where sg = 0;
                                aux1, aux2 both NULL or both set): with aux1 = s (the ∇-pass
                                adjoint), aux2 = u' = sg*z'/c2 and aux2_scale = beta*c2 this is
                                softplus' double-backward term beta*s*(1-sg)*z'  */
    CN_EPI_BWD_RELU = 6,     /* out0 = aux0 > 0 ? v : 0                              */
    CN_EPI_SOFTPLUS_HEAD = 8 /* the last SDF hidden layer with the sdf head fused (ABI v5):
                                a = softplus_beta(v + bias) (odiv 1); out0 = a (or NULL: not
                                stored); out1 = colv * sg(a) (or NULL: the ∇-pass seed
                                s = w80 ⊙ softplus', aux_beta > 0); head_out[head_idx ?
                                head_idx[m] : m] = Σ_n a[m][n] head_w[n] + head_b[0]
                                (neus_fields.py:279-283, the sdf column of lin8); needs the
                                whole row in one tile: N <= 256 (bf16x6) or N <= 128 */
} cn_epilogue;

typedef struct cn_linear_desc {
    const void* A;       /* fp32, or bf16 when a_bf16 (A2 likewise) */
    const void* A2;
    const float* B;
    const float* bias;   /* [N] or NULL (N <= 512 with a bias or colv) */
    const float* rowv;   /* [M] or NULL : rank-1 term rowv[m]*colv[n] added to v */
    const float* colv;   /* [N] or NULL */
    const void* aux0;    /* fp32, or bf16 when aux0_bf16 */
    const float* aux1;
    float* out0;
    float* out1;         /* SOFTPLUS_HEAD only (else NULL) */
    float* out_split;
    int64_t lda, lda2, ldb, ld_aux0, ld_aux1, ld_out0, ld_out1, ld_split;
    int32_t M, N, K, K1;
    int32_t nzero, nsplit;
    int32_t epilogue;    /* cn_epilogue */
    int32_t tile;        /* 0: the library's tile choice (up to 256x256), 1: 128x64, 2: 128x128 only
                            (tests compare the tiles: every tile gives the same bits) */
    float adiv, odiv;    /* divisors applied to A·Bᵀ and to the activation (0 means 1),
                            applied as multiplies by their fp32 reciprocals */
    float beta, threshold; /* Softplus(beta, threshold) of neus_fields.py:266 */
    int32_t mfma_dtype;  /* CN_MFMA_F32: A, B fp32, exact fp32 products (v_mfma_f32_32x32x2_f32);
                            CN_MFMA_BF16: A fp32 rounded to bf16 (RNE) on load, B bf16 [N][ldb]
                            (ldb in bf16 elements), fp32 accumulate (v_mfma_f32_32x32x16_bf16);
                            K and K1 multiples of 64 (config C3's bf16 MLP MFMA);
                            CN_MFMA_F32_BF16X6: fp32 GEMM on the bf16 MFMA: A fp32 split on load
                            into three bf16 terms, B pre-split and chunk-major: bf16
                            [K/16][ldb][3][16], term t of element (n, k) at
                            B + ((k/16) ldb + n) 48 + 16 t + k%16, ldb = image rows >= the N
                            tiles; six term products accumulated in fp32 (error at the level
                            of fp32 accumulation; K, K1 multiples of 32) */
    float aux_beta;      /* sg() scale of MUL / TANGENT / BWD_SOFTPLUS (> 0 for those) */
    const float* aux2;   /* BWD_SOFTPLUS second-order input u' (or NULL) */
    int64_t ld_aux2;
    float aux2_scale;
    int32_t flags;       /* bit 0: visit the M-tiles last to first (a chain's consecutive launches
                            alternate it so a layer first reads the rows its producer wrote last,
                            still in the memory-side cache); results do not depend on it */
    const float* head_w;       /* SOFTPLUS_HEAD: [N] row-dot weights, head_b: [1] */
    const float* head_b;
    float* head_out;           /* [M] (or indexed by head_idx) */
    const int32_t* head_idx;   /* [M] destination rows or NULL */
    /* ABI v10 -- bf16 operand images (CN_MFMA_BF16 only, config C3's bf16 MLP MFMA): a GEMM operand
       is rounded to bf16 (RNE) when it is staged, so a tensor whose consumers are GEMM operands can be
       stored as that rounded image (2 bytes instead of 4) with bitwise-identical results.
       a_bf16: A and A2 are bf16 row-major (lda / lda2 in bf16 elements, multiples of 8).
       aux0_bf16: aux0 is bf16 -- BWD_RELU's sign source (bf16 RNE keeps the sign, and a positive
       value rounds to 0 only below 2^-133), or the activation MUL / TANGENT / BWD_SOFTPLUS recover
       softplus' σ from (config C3 stores the SDF's hidden activations as bf16 images only; σ from
       the bf16 activation is within the mode's bf16 operand rounding).
       aux12_bf16: BWD_SOFTPLUS's aux1 and aux2 (the second-order term's s and u') are bf16 (config
       C3 stores the ∇-pass adjoints and the tangents, read only by GEMMs and by this term, in bf16).
       BWD_SOFTPLUS with aux1 / aux2 takes all three aux operands in one format: aux0_bf16 ==
       aux12_bf16.
       out0_b (ld_out0_b): the bf16 image of every value written to out0 (columns [0, nzero),
       including the zero fill); out0 itself may then be NULL.  out1_b: the same for SOFTPLUS_HEAD's
       out1 (colv and aux_beta set; out1 may then be NULL).  Leading dimensions in bf16 elements, multiples of 8; 16-byte aligned. */
    int32_t a_bf16;
    int32_t aux0_bf16;
    int32_t aux12_bf16;
    void* out0_b;
    int64_t ld_out0_b;
    void* out1_b;
    int64_t ld_out1_b;
} cn_linear_desc;

enum cn_mfma_dtype { CN_MFMA_F32 = 0, CN_MFMA_BF16 = 1, CN_MFMA_F32_BF16X6 = 2 };

int cn_linear(const cn_linear_desc* d, cn_stream_t stream);

/* The rocprofv3 symbol of the kernel cn_linear would launch for *d (no launch, no device
 * access; the tile choice is the launch's own function): NUL-terminated into buf[len].
 * Returns the name's length, or a negative cn_status.  For profilers and the bench's
 * roofline (bench.py names the launch class it reports). */
int cn_linear_kernel_name(const cn_linear_desc* d, char* buf, int32_t len);

/* ------------------------------------------------------------------------ *
 * Weight images for cn_linear (the per-call `pack` of the effective weights,
 * neus_fields.py:273-283 / 364-373 weight_norm outputs): one launch builds
 * every padded / transposed / column-permuted B image of a network.  Job j
 * writes the region [r0, r1) x [c0, c1) of its image: the source matrix
 * S (rows x cols; S[r][c] = src[r*src_ld + c], or src[c*src_ld + r] when
 * transpose) lands at (r0, c0), the rest of the region is zero.  format is a
 * cn_mfma_dtype: CN_MFMA_F32 copies fp32 (element (r, c) at dst[r*dst_ld + c]),
 * CN_MFMA_BF16 rounds to bf16 (RNE, same indexing), CN_MFMA_F32_BF16X6 writes
 * the three bf16 terms of each value into cn_linear's chunk-major image (term t
 * at dst[((c/16)*dst_ld + r)*48 + 16t + c%16]; dst_ld = the image's rows).
 * ------------------------------------------------------------------------ */
typedef struct cn_pack_job {
    const float* src;
    void* dst;
    int64_t src_ld, dst_ld;
    int32_t rows, cols;
    int32_t r0, r1, c0, c1;
    int32_t transpose;
    int32_t format;
} cn_pack_job;

int cn_pack_weights(const cn_pack_job* jobs, int32_t njobs, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Weight normalisation of every Linear of a network in one launch
 * (torch.nn.utils.weight_norm, dim 0, as the reference wraps every layer:
 * model/neus_fields.py:84-140, 336-360): per output row i,
 *   forward   W_i = v_i (g_i / |v_i|)
 *   backward  dg_i = (dW_i . v_i) / |v_i|,  dv_i = (g_i / |v_i|) (dW_i - v_i dg_i / |v_i|)
 * v, w, dw, dv row-major contiguous [rows][cols]; g, dg [rows].  One wavefront per
 * row (fixed-order reductions).
 * ------------------------------------------------------------------------ */
typedef struct cn_wn_job {
    const float* v;
    const float* g;
    float* w;            /* forward output */
    const float* dw;     /* backward input */
    float* dv;           /* backward outputs */
    float* dg;
    int32_t rows, cols;
} cn_wn_job;

int cn_weight_norm(const cn_wn_job* jobs, int32_t njobs, int32_t backward, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Weight gradient: dW[n][k] = sum_m ( Y0[m][n]*X0[m][k] + Y1[m][n]*X1[m][k] ),
 * db[n] = sum_m Y0[m][n].  Reduction over the M = R*S sample rows is split
 * over workgroups into fp32 slabs (workspace) and summed in a fixed order, so
 * the result is bitwise reproducible.  Replaces the dW/db of the autograd of
 * every Linear above, including the create_graph term of neus_fields.py:296.
 * ------------------------------------------------------------------------ */
typedef struct cn_wgrad_desc {
    const void* Y0;      /* fp32, or bf16 when y_bf16 (Y1 likewise) */
    const void* X0;      /* fp32, or bf16 when x_bf16 (X1 likewise) */
    const void* Y1;      /* NULL when npairs == 1 */
    const void* X1;
    float* workspace;    /* cn_wgrad_workspace_bytes() */
    float* dW;           /* [n_out][k_out] (ld_dw) */
    float* db;           /* [n_out] or NULL */
    int64_t ldy0, ldx0, ldy1, ldx1, ld_dw;
    int64_t workspace_bytes;
    int32_t M, N, K;     /* N, K: valid columns of Y and X (Y/X readable up to the padded tile) */
    int32_t npairs;
    int32_t n_out, k_out;
    int32_t accumulate;  /* 1: dW += result (db too), 0: dW = result */
    int32_t mfma_dtype;  /* CN_MFMA_F32, or CN_MFMA_BF16: Y and X rounded to bf16 (RNE) on load,
                            v_mfma_f32_32x32x16_bf16, fp32 accumulation and slab reduction;
                            db is summed from the fp32 values either way;
                            CN_MFMA_F32_BF16X6: fp32 gradient from three bf16 terms per operand
                            (six products) */
    /* ABI v10 (CN_MFMA_BF16 only): the Y side (Y0, Y1) / the X side (X0, X1) are bf16 operand images
       (see cn_linear_desc.a_bf16; leading dimensions in bf16 elements, multiples of 8): the products
       are the same bits as from the fp32 tensors they round; db then sums the bf16 values of Y0. */
    int32_t y_bf16;
    int32_t x_bf16;
} cn_wgrad_desc;

size_t cn_wgrad_workspace_bytes(int32_t M, int32_t N, int32_t K);
int cn_wgrad(const cn_wgrad_desc* d, cn_stream_t stream);
/* As cn_linear_kernel_name for cn_wgrad's split-M kernel (cn::slab_reduce_kernel follows it). */
int cn_wgrad_kernel_name(const cn_wgrad_desc* d, char* buf, int32_t len);
/* Several independent weight gradients (ABI v9).  The descriptors that cn_wgrad would run on a
 * 256x256 stage-ring kernel (bf16x6, or bf16 since ABI v10) share ONE launch of it (each takes a share of the workgroups
 * proportional to its rows x pairs x output tiles, its own M-slices and slabs in its own
 * workspace) and ONE cn::slab_reduce_kernel launch; any other descriptor is run as by cn_wgrad.
 * Results equal cn_wgrad's up to the slice count (fixed-order sums: bitwise reproducible).
 * Replaces the per-layer dW of neus_fields.py:291-303 (SDF) and 364-373 (colour) as one call. */
int cn_wgrad_batch(const cn_wgrad_desc* descs, int32_t n, cn_stream_t stream);
/* ABI v10: the workspace a cn_wgrad_batch call over descs[0..n) needs (n <= 64), and each
 * descriptor's byte offset into one buffer of that size (offsets may be NULL): a batched job takes
 * only its share of the slabs, so this is less than the sum of cn_wgrad_workspace_bytes.  The
 * layout follows the CU count of the current device: query and launch on the same device. */
size_t cn_wgrad_batch_workspace_bytes(const cn_wgrad_desc* descs, int32_t n, int64_t* offsets);

/* ------------------------------------------------------------------------ *
 * Per-row heads (neus_fields.py:279-283 last Linear row 0 = sdf;
 * neus_fields.py:367-373 last colour Linear + sigmoid):
 *   out[dst(m)][c] = act( sum_k A[m][k]*W[c][k] + b[c] ),  c < C (C <= 4)
 * act: 0 none, 1 sigmoid.  dst(m) = dst_index ? dst_index[m] : m.
 * ------------------------------------------------------------------------ */
int cn_row_head(int32_t M, int32_t K, const float* A, int64_t lda, const float* W, int64_t ldw,
                const float* b, int32_t C, int32_t act, float* out, int64_t ld_out,
                const int32_t* dst_index, cn_stream_t stream);

/* out[k] (+)= (sum_m (w ? w[m] : 1) * X[m][k]) / wdiv, k < K: the sdf row of the
 * last SDF Linear's weight gradient (neus_fields.py:283, row 0 of lin8) and its
 * create_graph term; fixed-order slab reduction. */
size_t cn_colsum_workspace_bytes(int32_t M, int32_t K);
int cn_colsum(int32_t M, int32_t K, const float* w, const float* X, int64_t ldx, float wdiv, float* out,
              int32_t accumulate, float* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* out[m][n] = f(X[m][n]) * w[n] (* rowv[m] when rowv != NULL) for n < N: the seed of the
 * ∇ₓSDF pass (neus_fields.py:295-302), and the sdf-only adjoint of the last hidden layer
 * (d sdf / d z_7 = dsdf[m] w80[n] softplus'(z_7), no feature gradient: no GEMM needed);
 * f(x) = x when act_beta == 0, else softplus' from the softplus output, 1 - exp(-act_beta x). */
int cn_scale_cols(int32_t M, int32_t N, const float* X, int64_t ldx, const float* w, const float* rowv,
                  float* out, int64_t ld_out, float act_beta, cn_stream_t stream);

/* Adjoint of a softplus layer from the gradient of its output, without a GEMM (the
 * SDF's last hidden layer when the feature head is folded into the colour network's
 * first layer: the colour backward already yields d/d(hidden)):
 *   out[m][n] = ((D ? D[m][n] : 0) + (rowv ? rowv[m] colv[n] : 0)) * sg
 *             + (aux1 ? aux1[m][n] aux2[m][n] aux2_scale (1 - sg) / sg : 0),   0 where sg = 0,
 *   sg = 1 - exp(-act_beta act[m][n]) (softplus' from the activation, as cn_linear's epilogues). */
/* With cs_out != NULL it also produces the sdf row of lin8's weight gradient from the
 * operands it already streams (the fused form of cn_colsum's calls):
 *   cs_out[n] = (sum_m (rowv ? rowv[m] act[m][n] : 0) + (aux2 ? aux2[m][n] : 0)) / cs_div,
 *   rs_out[0] = (sum_m rowv[m]) / cs_div (the sdf head's bias gradient; rs_out may be NULL),
 * fixed-order slab reductions through workspace (cn_softplus_adjoint_workspace_bytes). */
size_t cn_softplus_adjoint_workspace_bytes(int32_t M, int32_t N);
/* out_bf16 (ABI v10): out is written as its bf16 operand image (RNE; ld_out in bf16 elements, % 4 == 0).
 * in_bf16 (ABI v10): bit 0: D, bit 1: act, bit 2: aux1 and aux2 are bf16 operand images (config C3's
 * bf16 mode; leading dimensions in bf16 elements, % 4 == 0, 8-byte aligned). */
int cn_softplus_adjoint(int32_t M, int32_t N, const void* D, int64_t ldd, const void* act, int64_t lda,
                        float act_beta, const float* rowv, const float* colv, const void* aux1, int64_t ld1,
                        const void* aux2, int64_t ld2, float aux2_scale, void* out, int64_t ld_out, int32_t out_bf16,
                        int32_t in_bf16, float* cs_out, float* rs_out, float cs_div, float* workspace,
                        int64_t workspace_bytes, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Positional encoding of the SDF input (neus_embedder.py:6-51 with
 * include_input, log-sampled bands 2^0..2^(multires-1), [sin, cos]; applied at
 * neus_fields.py:269-271 to x*scale):
 *   U0[m][0..4+8*multires) = embed(scale * x[m][0..4)),  zeros up to kpad.
 *   If U4e != NULL also U4e[m][j] = U0[m][j] / u4_scale (the skip-connection
 *   copy of neus_fields.py:276-277).  flags bit 0 (ABI v10): U4e is a bf16
 *   operand image (RNE; ld_u4 in bf16 elements, 8-byte aligned); bit 1 (ABI
 *   v11): U0 is one too (the operand of cn_sdf_mlp; 8-byte aligned).
 * ------------------------------------------------------------------------ */
int cn_sdf_embed(int32_t M, const float* x, int64_t ldx, int32_t multires, float scale, int32_t kpad,
                 void* U0, int64_t ld_u0, void* U4e, int64_t ld_u4, float u4_scale, int32_t flags,
                 cn_stream_t stream);

/* ∇ₓSDF from the embedding adjoint: G[m][i] = scale * J_embed(x)ᵀ (Q0[m] + QE[m])
 * (neus_fields.py:291-303; the chain rule through neus_embedder.py:20-22). */
int cn_sdf_grad_assemble(int32_t M, int32_t multires, float scale, const float* U0, int64_t ld_u0,
                         const float* Q0, int64_t ld_q0, const float* QE, int64_t ld_qe,
                         float* G, int64_t ld_g, cn_stream_t stream);

/* Tangent of the embedding along v = dL/d(∇ₓSDF) (forward-over-reverse form
 * of the double backward of neus_fields.py:296):
 *   T0[m] = scale * J_embed(x) v[m] (zeros up to kpad);  T4e[m] = T0[m] / t4_scale
 *   (t4_bf16, ABI v10: T4e a bf16 operand image, as cn_sdf_embed's U4e). */
int cn_sdf_tangent_prep(int32_t M, int32_t multires, float scale, int32_t kpad, const float* U0,
                        int64_t ld_u0, const float* v, int64_t ld_v, float* T0, int64_t ld_t0,
                        void* T4e, int64_t ld_t4, float t4_scale, int32_t t4_bf16, cn_stream_t stream);

/* Colour-network input extras (neus_fields.py:346-356, mode 'idr'):
 *   ext[m] = [ G[m][0..4), pts[m][0..4), embed_view(dirs[m / dir_div]) (3+6*multires_view), 0... ]
 * The 256 feature columns are read in place by cn_linear through A/A2. */
int cn_color_extras(int32_t M, const float* G, int64_t ld_g, const float* pts, int64_t ld_p,
                    const float* dirs, int64_t ld_d, int32_t dir_div, int32_t multires_view,
                    int32_t kpad, float* ext, int64_t ld_ext, cn_stream_t stream);

/* Ray-direction gradient through the view encoding of cn_color_extras (the
 * autograd of neus_embedder.py:17-36 on dirs, neus_renderer.py:345, 354):
 * with d_ext [M][>=8+3+6L] the gradient of ext, rows r*dir_div .. r*dir_div +
 * dir_div-1 sharing dirs[r],
 *   ddirs[r][c] (+)= sum_rows d_ext[.][8+c]
 *                  + sum_k 2^k (cos(2^k d_c) d_ext[.][11+6k+c] - sin(2^k d_c) d_ext[.][14+6k+c]). */
int cn_color_extras_bwd(int32_t R, int32_t dir_div, const float* d_ext, int64_t ld_ext, const float* dirs,
                        int64_t ld_d, int32_t multires_view, float* ddirs, int32_t accumulate,
                        cn_stream_t stream);

/* Backward of the colour head (sigmoid(Linear 256->3), neus_fields.py:367-373):
 *   dz3 = drgb*rgb*(1-rgb);  dZ2[m][k] = (H3[m][k] > 0) * sum_c dz3[m][c]*W3[c][k];
 *   dW3 = sum_m dz3ᵀ H3, db3 = sum_m dz3 (fixed-order slab reduction). */
size_t cn_rgb_head_bwd_workspace_bytes(int32_t M, int32_t K);
int cn_rgb_head_bwd(int32_t M, int32_t K, const float* drgb, const float* rgb, const float* H3,
                    int64_t ld_h, const float* W3, void* dZ2, int64_t ld_dz, int32_t dz_bf16, float* dW3,
                    float* db3, float* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Patch sampling (model/training.py:413-436 on the device): idx[p*ps*ps + a*ps + b] =
 * (row_p + a) * w + col_p + b for n_patches distinct corners (row_p, col_p) of the
 * (h-ps+1) x (w-ps+1) grid -- the first n_patches values of a keyed pseudo-random
 * permutation of the corner ids (4-round Feistel network with cycle walking; key:
 * 4 int32 on the device, e.g. from torch.randint), the device counterpart of
 * randperm(n)[:n_patches] without a sort.
 * ------------------------------------------------------------------------ */
int cn_patch_indices(int32_t h, int32_t w, int32_t ps, int32_t n_patches, const int32_t* key, int64_t* idx,
                     cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Stage-1 relative poses (neus_fields.py:142-161, every interval at once): for
 * interval k < K with its n time steps, A_s = EulerXYZ(omega_s dt_k) (pytorch3d
 * convention, Rx Ry Rz), V_s = vel_s dt_k, T <- A_s T + V_s, Q <- Q A_s from
 * Q = I, T = 0; P[k] = [Q T; 0 0 0 1] (row-major 4x4).  omega / vel rows
 * k*n + s with leading dimensions ld_o / ld_v (floats).  The backward maps dP
 * [K][4][4] to domega, dvel ([K*n][3] contiguous) by the reverse recurrence.
 * One thread per interval (n <= 64).
 * ------------------------------------------------------------------------ */
int cn_euler_chain(int32_t K, int32_t n, const float* omega, int64_t ld_o, const float* vel, int64_t ld_v,
                   const float* dt, float* P, cn_stream_t stream);
int cn_euler_chain_bwd(int32_t K, int32_t n, const float* omega, int64_t ld_o, const float* vel, int64_t ld_v,
                       const float* dt, const float* dP, float* domega, float* dvel, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Sampling along rays (neus_renderer.py:453-525).
 * ------------------------------------------------------------------------ */
/* Uniform jitter from a counter-based generator (ABI v14; the §8(b) device Philox seed): out[i] =
 * (word i % 4 of Philox4x32-10(counter = (i / 4 as 64 bits, offset), key = seed)) >> 8, x 2^-24, in [0, 1).
 * seed_offset: DEVICE uint64 [2] = (seed, offset), read by the kernel, so a captured launch replays with
 * the current values (the caller advances offset by ceil(n / 4) per draw to keep streams disjoint). */
int cn_uniform_philox(int64_t n, const uint64_t* seed_offset, float* out, cn_stream_t stream);

/* z[r][i] = near*(1-lin_i) + far*lin_i, lin = linspace(0,1,n); stratified
 * jitter with t_rand [R][n] when t_rand != NULL (neus_renderer.py:466-483). */
int cn_coarse_z(int32_t R, int32_t n, const float* near, const float* far, const float* t_rand,
                float* z, cn_stream_t stream);

/* pts_time[r*n+i] = [o_r + d_r * zz_i, t]: zz = z (mid == 0) or the section
 * midpoints z + dists/2 with the last dist = (far[0]-near[0])/n_coarse
 * (neus_renderer.py:337-350, 495-498, 286-291). */
int cn_points(int32_t R, int32_t n, const float* rays_o, const float* rays_d, const float* z,
              const float* t, int32_t mid, const float* near, const float* far, int32_t n_coarse,
              float* pts_time, cn_stream_t stream);

/* Backward of cn_points for ray / pose gradients (the autograd of
 * neus_renderer.py:343-350, pts = rays_o + rays_d * mid_z): with dP [R*n][>=3]
 * (row stride ld_p) the upstream gradient of pts_time,
 *   drays_o[r] = sum_i dP[r*n+i][0..3),  drays_d[r] = sum_i dP[r*n+i][0..3) * zz_i
 * (zz as in cn_points).  One wavefront per ray, fixed-order double sums. */
int cn_points_bwd(int32_t R, int32_t n, const float* z, int32_t mid, const float* near, const float* far,
                  int32_t n_coarse, const float* dP, int64_t ld_p, float* drays_o, float* drays_d,
                  cn_stream_t stream);

/* One NeuS up-sampling round + merge (neus_renderer.py:178-224 up_sample,
 * 39-70 sample_pdf det=True, 282-298 cat_z_vals).  One wavefront per ray.
 *   z_out = sorted merge of z and the n_imp new samples;
 *   z_new = the new samples [R][n_imp];
 *   if sdf_out: sdf_out[r][pos(old i)] = sdf[r][i] and new_dst[r*n_imp+j] =
 *   r*(n+n_imp) + pos(new j) (cn_row_head scatters the new SDF there). */
int cn_up_sample_merge(int32_t R, int32_t n, int32_t n_imp, float inv_s, const float* z,
                       const float* sdf, float* z_out, float* z_new, float* sdf_out, int32_t* new_dst,
                       cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Alpha compositing (neus_renderer.py:337-420, render_core).  One wavefront
 * per ray; transmittance as an exclusive product scan across the wave.
 * G holds ∇ₓSDF rows (normals = G[m][0..3)), sdf/G/rgb are indexed m = r*S+i.
 * inv_s and cos_anneal_ratio are device scalars (training.py:120-124 ramps the
 * ratio every iteration: a replayed hipGraph reads the current value). 
 * ------------------------------------------------------------------------ */
int cn_composite_fwd(int32_t R, int32_t S, const float* z, const float* sdf, const float* G,
                     int64_t ld_g, const float* rgb, const float* rays_d, const float* inv_s,
                     const float* near, const float* far, int32_t n_coarse, const float* cos_anneal_ratio,
                     float* color, float* depth, float* weights, float* cdf, cn_stream_t stream);

/* Backward of cn_composite_fwd.  drays_d (nullable, [R][3]) receives the ray
 * direction gradient of true_cos = rays_d . normals (neus_renderer.py:362);
 * the normals are those of the detached-input gradient pass
 * (neus_renderer.py:356), so no second-order term reaches the points. */
int cn_composite_bwd(int32_t R, int32_t S, const float* z, const float* sdf, const float* G,
                     int64_t ld_g, const float* rgb, const float* rays_d, const float* inv_s,
                     const float* near, const float* far, int32_t n_coarse, const float* cos_anneal_ratio,
                     const float* dcolor, const float* ddepth, const float* dweights,
                     const float* dcdf, float* dsdf, float* dG, float* drgb, float* dinv_s_part,
                     float* drays_d, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Training losses in one pass: the loss value and its input gradients
 * (model/training.py:506-509 colour L1, train.py:526 eikonal, model/losses.py:7-38
 * with train.py:519-525 edge-aware and plain depth smoothness on patch x patch
 * ray patches, patch in 1..4; R rays, M samples):
 *   loss = w_rgb sum|color - gt| / R + w_eik mean_m (|n_m| - 1)^2
 *        + w_edge EdgePreservingSmoothness(depth, gt; gamma) + w_smooth Smoothness(depth)
 *   weights: DEVICE [4] = (w_rgb, w_eik, w_edge, w_smooth), read by the kernels, so the
 *   annealed weights of train.py:246-263, 401-405 change without re-capturing a graph;
 *   nonfinite (nullable, device int32): set to 1 when the loss is not finite -- the
 *   NaN assert of model/training.py:532-533 without a host sync;
 *   color, gt [R][3]; depth [R]; normals [M][ld_n] (columns 0..2); loss [1];
 *   dcolor [R][3], ddepth [R], dnormals [M][ld_dn] (columns 0..2) = d loss / d input.
 * Partial sums are reduced in double in a fixed order (bitwise reproducible).
 * ------------------------------------------------------------------------ */
size_t cn_train_loss_workspace_bytes(int32_t R, int32_t patch);
int cn_train_loss(int32_t R, int32_t patch, int64_t M, const float* color, const float* gt, const float* depth,
                  const float* normals, int64_t ld_n, const float* weights, float gamma, float* loss,
                  float* dcolor, float* ddepth, float* dnormals, int64_t ld_dn, int32_t* nonfinite,
                  void* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Stage-1 per-sample terms (train.py:467-505), R rays of S samples, M = R*S,
 * in one pass each way (replaces the ~40 torch ops of train.py:468-477, the
 * per-ray sums the flow projection reduces to (train.py:484-495) and the
 * point transform of the SDF-consistency term (train.py:502-504)):
 *   pts [M][ld_p], normals [M][ld_n] (columns 0..2), flows [M] (stride ld_f),
 *   weights [R][S]; mv: DEVICE [6] = (angular_velocity, velocity);
 *   cw2: DEVICE [4][4] (row-major) or null -- camera-of-frame -> world-camera;
 * forward:
 *   sums [2]       = (sum_m |(w x p_m + v) . n_m + f_m| w_m, sum_m w_m)
 *   ray_acc [R][4] = (sum_s w p, sum_s w) per ray (16B aligned)
 *   x_out [M][ld_x] (nullable, needs cw2) = (cw2 (p_m, 1))[0..2], t_world
 * backward (g_num: DEVICE [1] = dL/d sums[0]; the weights are detached there,
 * as in the reference; d_ray [R][4] and dx [M][ld_dx] (columns 0..2) nullable):
 *   dnormals [M][ld_dn], dflows [M] (stride ld_df): written;
 *   dweights [R][S] (nullable) = d_ray . (p, 1);
 *   dpts [M][ld_dp] (nullable): written;
 *   dmv_dcw2 [18] = (dL/d mv [6], dL/d cw2 rows 0..2 [12]).
 * The cross-ray sums are per-workgroup partials reduced in a fixed order
 * (bitwise reproducible); workspace: cn_stage1_workspace_bytes(R).
 * ------------------------------------------------------------------------ */
size_t cn_stage1_workspace_bytes(int32_t R);
int cn_stage1_fwd(int32_t R, int32_t S, const float* pts, int64_t ld_p, const float* normals, int64_t ld_n,
                  const float* flows, int64_t ld_f, const float* weights, const float* mv, const float* cw2,
                  float t_world, float* ray_acc, float* x_out, int64_t ld_x, float* sums, float* workspace,
                  cn_stream_t stream);
int cn_stage1_bwd(int32_t R, int32_t S, const float* pts, int64_t ld_p, const float* normals, int64_t ld_n,
                  const float* flows, int64_t ld_f, const float* weights, const float* mv, const float* cw2,
                  const float* g_num, const float* d_ray, const float* dx, int64_t ld_dx, float* dnormals,
                  int64_t ld_dn, float* dflows, int64_t ld_df, float* dweights, float* dpts, int64_t ld_dp,
                  float* dmv_dcw2, float* workspace, cn_stream_t stream);

/* Running products of n 4x4 matrices (row-major [n][4][4]), ABI v8: C_0 = A_0,
 * C_j = A_j C_{j-1} -- the relative-pose chains of stage 1 (compute_w2c_mappings,
 * model/neus_fields.py:171-183; the world-camera chain of train.py:498-501) -- and the
 * adjoint: dA from dC (every C_j may carry a gradient).  One lane walks the chain. */
int cn_mat4_chain_fwd(int32_t n, const float* A, float* C, cn_stream_t stream);
int cn_mat4_chain_bwd(int32_t n, const float* A, const float* C, const float* dC, float* dA, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * The sampler's SDF query in one launch (ABI v11): SDFNetwork.sdf(x) with no
 * gradient, as NeuSRenderer.up_sample calls it (model/neus_renderer.py:492-525,
 * the coarse samples and each round's new ones; neus_fields.py:268-283) -- eight
 * softplus layers with the skip concat and the sdf row of the last Linear -- for
 * the bf16 MLP MFMA mode (config C3), from the embedding's bf16 images that
 * cn_sdf_embed writes (flags 3).  Activations stay on chip: per sample 128 + 2E
 * bytes are read and the sdf (4 B) written.  Bitwise equal to the
 * layer-by-layer bf16 path (cn_linear on bf16 weight images, SOFTPLUS /
 * SOFTPLUS_HEAD epilogues).
 *   u0      [M][ld_u0] bf16: the embedding, 64 columns (lin0's input; zero past E),
 *           ld_u0 % 8 == 0, 16-byte aligned;
 *   tail    [M][ld_t] bf16: the embedding / skip_div, E = 4 (1 + 2 multires)
 *           columns (the skip concat's tail), ld_t % 4 == 0, 8-byte aligned;
 *   W[l]    bf16 weight images [256][ldw[l]] of lin0 .. lin7, K = 64 (lin0) or 256,
 *           rows past a layer's width zero (as cn_pack_weights builds them);
 *   bias[l] fp32 [width]; the skip layer (feeding the skip concat) has width
 *           256 - E, its output divided by skip_div;
 *   head_w  [256] = lin8.weight[0] / scale, head_b [1] = lin8.bias[0] / scale;
 *   sdf     written at idx[m] (idx NULL: m).
 * Supported: n_layers 8, hidden 256, kpad0 64, multires <= 7; else
 * CN_ERR_UNSUPPORTED (the caller composes cn_linear launches instead).
 * ------------------------------------------------------------------------ */
typedef struct cn_sdf_mlp_desc {
    const void* u0;   /* bf16 */
    const void* tail; /* bf16 */
    int64_t ld_u0, ld_t;
    int32_t M, n_layers, hidden, kpad0, multires, skip_layer;
    const void* W[8]; /* bf16 */
    int64_t ldw[8];
    const float* bias[8];
    const float* head_w;
    const float* head_b;
    float* sdf;
    const int32_t* idx;
    float skip_div, beta, threshold;
    void* debug; /* NULL, or [8][M][256] (bf16; fp32 in the bf16x6 format): every layer's input as the kernel holds it (tests) */
    int32_t format; /* 0: the bf16 mode (u0 / tail bf16 images, W bf16 [256][K]); CN_MFMA_F32_BF16X6 (ABI v15): the
                       fp32-class mode -- u0 / tail fp32, W the chunk-major term images [K/16][256][48] of
                       cn_pack_weights (ldw = 256, their rows), bitwise the layer-by-layer bf16x6 query */
} cn_sdf_mlp_desc;
int cn_sdf_mlp(const cn_sdf_mlp_desc* d, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Composed entry points (ABI v12): the sampler of NeuSRenderer.render
 * (neus_renderer.py:466-525) and the SDF query it makes (SDFNetwork.sdf,
 * neus_fields.py:268-283, 286-287), each one C call over the kernels above --
 * no host code between the launches, all on the caller's stream, scratch from
 * a caller-owned workspace (size from the *_workspace_bytes function; 256-byte
 * aligned; it may be reused as soon as the stream has passed the call).
 * Results are bitwise those of the same kernels composed one by one
 * (copenerf.fields.sdf_forward / copenerf.renderer.sample_z).
 *
 * cn_sdf_net describes SDFNetwork's weights as cn_pack_weights images
 * (copenerf.fields.pack_sdf): for lin0 .. lin(n_lin-2) the forward image
 * W[l] (rows w_rows[l] >= the output width rounded up to 128, columns w_cols[l]:
 * KE = 64-rounded encoding width for lin0, the 32- (bf16: 64-) rounded input
 * width after; CN_MFMA_F32_BF16X6 images are chunk-major [w_cols/16][w_rows][48]),
 * bias[l] fp32 [out_dim[l]] (16-byte aligned); the sdf row of the last Linear
 * as head_w [in_dim[n_lin-1]] = weight[0] / scale (16-byte aligned) and head_b
 * [1] = bias[0] / scale.  skip: the layer whose input is cat([h, embed(x)]) / sqrt 2
 * (SDFNetwork skip_in, one entry) or -1; the layer before it has width
 * out_dim = d_hidden - E.  Inputs are (x, y, z, t) points (d_in = 4), E = 4 (1 + 2 multires).
 * flags bit 0 (CN_SDF_LAYERED): never the fused cn_sdf_mlp query (tests compare the two).
 * ------------------------------------------------------------------------ */
#define CN_SDF_MAX_LIN 16
#define CN_SDF_LAYERED 1
typedef struct cn_sdf_net {
    int32_t n_lin;                      /* Linear layers (SDFNetwork n_layers + 1), 2 .. 16 */
    int32_t in_dim[CN_SDF_MAX_LIN];     /* lin_l.weight.shape[1] */
    int32_t out_dim[CN_SDF_MAX_LIN];    /* lin_l.weight.shape[0] */
    int32_t skip;
    int32_t multires;
    float scale, beta, threshold;       /* SDFNetwork scale, Softplus(beta, threshold) */
    int32_t mfma_dtype;                 /* cn_mfma_dtype of the images */
    int32_t flags;
    const void* W[CN_SDF_MAX_LIN - 1];
    int32_t w_rows[CN_SDF_MAX_LIN - 1];
    int32_t w_cols[CN_SDF_MAX_LIN - 1];
    const float* bias[CN_SDF_MAX_LIN - 1];
    const float* head_w;
    const float* head_b;
    /* ABI v13 (cn_render_fwd's ∇ₓSDF pass only): the transposed images Wt[l] (fields.pack_sdf's Bt:
       rows >= the input width rounded up to 128, columns the output width rounded up to 32 / 64) and
       head_wp [HL] = head_w zero-padded to the hidden buffers' width (16-byte aligned) */
    const void* Wt[CN_SDF_MAX_LIN - 1];
    int32_t wt_rows[CN_SDF_MAX_LIN - 1];
    int32_t wt_cols[CN_SDF_MAX_LIN - 1];
    const float* head_wp;
} cn_sdf_net;

/* sdf[idx ? idx[m] : m] = SDFNetwork.sdf(x[m]) for M points x [M][ldx >= 4] (no gradient):
 * cn_sdf_embed + cn_sdf_mlp (bf16 images, the fused shape) or cn_sdf_embed + one cn_linear per
 * layer (SOFTPLUS, the last with the SOFTPLUS_HEAD epilogue where one tile spans the row) +
 * cn_row_head otherwise. */
size_t cn_sdf_query_workspace_bytes(const cn_sdf_net* net, int32_t M);
int cn_sdf_query(const cn_sdf_net* net, int32_t M, const float* x, int64_t ldx, float* sdf,
                 const int32_t* idx, void* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* The sampler: z [R][n_samples + up_sample_steps k] (k = n_importance / up_sample_steps >= 1, or
 * [R][n_samples] when n_importance == 0) = the coarse samples (stratified with
 * t_rand [R][n_samples], or none when t_rand is NULL -- eval) and, when n_importance > 0,
 * up_sample_steps rounds of k new samples each, round i with
 * inv_s = 64 * 2^i from the SDF of the current samples (the coarse SDF query, then one query per
 * round's new samples scattered into the merged order; no query after the last round).
 * rays_o / rays_d [R][3], near / far [R], time_step [1] (the frame's time value; points are
 * (o + d z, t)).  The caller picks n_samples / n_importance by the iteration (the
 * importance_sampling_start switch of neus_renderer.py:455-459). */
typedef struct cn_sample_desc {
    int32_t R, n_samples, n_importance, up_sample_steps;
    const float* rays_o;
    const float* rays_d;
    const float* near;
    const float* far;
    const float* t_rand;
    const float* time_step;
    const cn_sdf_net* net;
    float* z;
    /* ABI v14: with t_rand NULL and philox != NULL (DEVICE uint64 [2] = (seed, offset)), the jitter is
       drawn on the device: t_rand = cn_uniform_philox(R n_samples, philox) in the workspace */
    const uint64_t* philox;
} cn_sample_desc;
size_t cn_sample_workspace_bytes(const cn_sample_desc* d);
int cn_sample(const cn_sample_desc* d, void* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * The rendering forward in one call (ABI v13): NeuSRenderer.forward of the
 * eval path (neus_renderer.py:453-584 with render_core 307-450, no gradient):
 * the sampler (cn_sample, or the caller's z), the section midpoints, the SDF
 * field with its ∇ₓSDF pass and the feature head folded into the colour
 * network (copenerf.renderer's fold: the colour network's first layer reads
 * the SDF's last hidden activation), the colour network, the compositing.
 * Bitwise equal to copenerf's renderer with the same packs.
 *
 * cn_color_net: RenderingNetwork (mode idr, squeeze_out) as its images
 * (copenerf.fields.pack_color with the folded first layer): W[0] is lin0's
 * image over [feature (F) | gradient | pts | emb(dirs) | 0] (K = F + KX,
 * KX = 64-rounded 4 + 4 + 3 (1 + 2 multires_view)), W[l] the hidden layers';
 * head_w [3][in_dim[n_lin-1]] fp32 and head_b [3] the sigmoid head.
 * ------------------------------------------------------------------------ */
typedef struct cn_color_net {
    int32_t n_lin;                      /* Linear layers, 2 .. 16 */
    int32_t in_dim[CN_SDF_MAX_LIN];
    int32_t out_dim[CN_SDF_MAX_LIN];
    int32_t d_feature, multires_view;
    int32_t mfma_dtype;
    const void* W[CN_SDF_MAX_LIN - 1];
    int32_t w_rows[CN_SDF_MAX_LIN - 1];
    int32_t w_cols[CN_SDF_MAX_LIN - 1];
    const float* bias[CN_SDF_MAX_LIN - 1];
    const float* head_w;
    const float* head_b;
    /* ABI v14 (cn_render_bwd only): the transposed images of the backward (copenerf.fields.pack_color):
       Wt[l] for the hidden layers l >= 1 (rows >= the input width rounded up to 128, columns the output
       width rounded up to 32 / 64); lin0's feature columns transposed Wtf; its gradient columns
       transposed Wg [4][wg_ld] fp32; its extras columns [g | pts | emb(dirs)] transposed Wxt (rows 64). */
    const void* Wt[CN_SDF_MAX_LIN - 1];
    int32_t wt_rows[CN_SDF_MAX_LIN - 1];
    int32_t wt_cols[CN_SDF_MAX_LIN - 1];
    const void* Wtf;
    int32_t wtf_rows, wtf_cols;
    const float* Wg;
    int32_t wg_ld;
    const void* Wxt;
    int32_t wxt_rows, wxt_cols;
} cn_color_net;

/* z_in: [R][S] sample positions (the renderer's z_vals hook), or NULL: cn_sample's
 * (t_rand as there; NULL: eval).  inv_s, cos_anneal_ratio: device scalars [1].
 * Outputs (all required): z [R][S] (S = n_samples + up_sample_steps k, or z_in's S),
 * pts [R S][4] (the midpoints, (x, t)), sdf [R S], grad [R S][4] (∇ₓSDF: normals and the
 * sdf flow), rgb [R S][3], color [R][3], depth [R] (weighted z), weights [R][S], cdf [R][S]. */
typedef struct cn_render_desc {
    int32_t R, n_samples, n_importance, up_sample_steps, S_in;
    const float* rays_o;
    const float* rays_d;
    const float* near;
    const float* far;
    const float* t_rand;
    const float* time_step;
    const float* z_in;
    const float* inv_s;
    const float* cos_anneal_ratio;
    const cn_sdf_net* sdf_net;
    const cn_color_net* color_net;
    float* z;
    float* pts;
    float* sdf;
    float* grad;
    float* rgb;
    float* color;
    float* depth;
    float* weights;
    float* cdf;
    const uint64_t* philox;             /* ABI v14: as cn_sample_desc.philox (the sampler's jitter) */
} cn_render_desc;
size_t cn_render_fwd_workspace_bytes(const cn_render_desc* d);
int cn_render_fwd(const cn_render_desc* d, void* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * The rendering step under autograd (ABI v14): render_core of NeuSRenderer.forward
 * (neus_renderer.py:307-450) at given samples, with everything its backward needs kept
 * in the caller's `state` buffer, and the backward in one call.
 * cn_render_train_fwd takes the descriptor of cn_render_fwd with z_in required (the
 * samples: cn_sample's, drawn without gradient as in the reference) and writes pts, sdf,
 * grad, color, depth, weights, cdf (rgb, z unused: the colour values stay in the state);
 * z_in, rays, near / far, time_step, inv_s, cos_anneal_ratio, the networks and those
 * outputs must stay unchanged until cn_render_bwd has run.
 * cn_render_bwd takes the gradients of the outputs (NULL: none) and writes
 *   the SDF network's effective-weight gradients sdf_dW[l] [out][in] / sdf_db[l]
 *     (the last Linear's feature rows zero: the colour network's folded lin0 carries them),
 *   the colour network's col_dW[l] / col_db[l] (lin0 over the folded input in the
 *     reference column order [pts | emb(dirs) | gradient | feature]),
 *   dinv_s [R] (per-ray parts of dL/d inv_s; the caller sums them),
 *   drays_o / drays_d [R][3] (both or neither: the pose gradient through the points,
 *     the view directions and the compositing's cosine).
 * Gradients that reach one buffer from several consumers are summed in the order
 * autograd sums them for copenerf's composition (the sdf / ∇ₓSDF / point outputs' own
 * consumers first, then the compositing's, then the colour network's, then the SDF
 * network's), so the results are bitwise those of the composition
 * (copenerf.renderer with RENDER_NATIVE off).  state: cn_render_state_bytes; workspace:
 * cn_render_bwd_workspace_bytes (pose or not); both 256-byte aligned.
 * ------------------------------------------------------------------------ */
typedef struct cn_render_grads {
    const float* dcolor;                /* [R][3] */
    const float* ddepth;                /* [R] */
    const float* dweights;              /* [R][S] */
    const float* dcdf;                  /* [R][S] */
    const float* dsdf;                  /* [R S] */
    const float* dgrad;                 /* [R S][4] */
    const float* dpts;                  /* [R S][4] */
    float* sdf_dW[CN_SDF_MAX_LIN];
    float* sdf_db[CN_SDF_MAX_LIN];
    float* col_dW[CN_SDF_MAX_LIN];
    float* col_db[CN_SDF_MAX_LIN];
    float* dinv_s;
    float* drays_o;
    float* drays_d;
} cn_render_grads;
size_t cn_render_state_bytes(const cn_render_desc* d);
size_t cn_render_bwd_workspace_bytes(const cn_render_desc* d, int32_t pose);
int cn_render_train_fwd(const cn_render_desc* d, void* state, int64_t state_bytes, cn_stream_t stream);
int cn_render_bwd(const cn_render_desc* d, const cn_render_grads* g, const void* state, int64_t state_bytes,
                  void* workspace, int64_t workspace_bytes, cn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * The SDF query under autograd (ABI v14): SDFNetwork.sdf(x) with gradients to the
 * network's parameters and to x -- the stage-1 consistency re-query of
 * train.py:502-505 (neus_fields.py:268-283 and its autograd backward; the §8(b)
 * cn_mlp_fwd / cn_mlp_bwd) -- as two calls.  cn_mlp_fwd writes sdf [M] and keeps the
 * layer activations in the caller's `state` buffer (cn_mlp_state_bytes; unchanged until
 * cn_mlp_bwd has run).  cn_mlp_bwd takes dsdf [M] = dL/dsdf and that state and writes
 *   dW[l] [out_dim[l]][in_dim[l]] (row-major) and db[l] [out_dim[l]], l = 0 .. n_lin-1:
 *     the gradients of the effective weights (weight-norm's backward stays the caller's);
 *     the last Linear's rows past the sdf row (the feature head, unused by sdf()) are zero;
 *   dx [M][4] (16-byte aligned) = dL/dx when dx != NULL;
 *   dW[0] == NULL: dx only, no parameter gradients.
 * The network needs the transposed images (Wt, head_wp; cn_sdf_net ABI v13).  Scratch
 * from workspace (cn_mlp_bwd_workspace_bytes); state and workspace 256-byte aligned.
 * Bitwise equal to copenerf.fields.sdf_forward (keep) and sdf_backward (sdf only, first
 * order) / sdf_input_grad with the same packs.  M = 0: nothing is written.
 * ------------------------------------------------------------------------ */
typedef struct cn_mlp_desc {
    int32_t M;
    const float* x;                     /* [M][4] (x, y, z, t) -- cn_mlp_fwd */
    const cn_sdf_net* net;
    float* sdf;                         /* [M] -- cn_mlp_fwd */
    const float* dsdf;                  /* [M] -- cn_mlp_bwd */
    float* dW[CN_SDF_MAX_LIN];
    float* db[CN_SDF_MAX_LIN];
    float* dx;
} cn_mlp_desc;
size_t cn_mlp_state_bytes(const cn_mlp_desc* d);
size_t cn_mlp_bwd_workspace_bytes(const cn_mlp_desc* d);
int cn_mlp_fwd(const cn_mlp_desc* d, void* state, int64_t state_bytes, cn_stream_t stream);
int cn_mlp_bwd(const cn_mlp_desc* d, const void* state, int64_t state_bytes, void* workspace,
               int64_t workspace_bytes, cn_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* COPENERF_H_ */
