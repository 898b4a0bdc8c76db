// cn_pipeline.hip — composed entry points (ABI v12): the sampler's SDF query and the whole
// sampler of NeuSRenderer.render as single C calls over the kernels of this library.
//
// Reference: neus_renderer.py:466-525 (coarse z, up_sample rounds, cat_z_vals with the new
// samples' SDF) and neus_fields.py:268-283 / 286-287 (SDFNetwork.forward / .sdf).  The
// composition follows copenerf.fields.sdf_forward (want_feat=False, no gradient) and
// copenerf.renderer.sample_z launch for launch, so the results are the same bits; host code
// only plans buffers in the caller's workspace and fills descriptors -- nothing synchronises,
// allocates or touches the default stream, so a caller may capture cn_sample in a hipGraph.
#include <cmath>

#include "cn_common.h"

namespace {

constexpr size_t kAlign = 256;

size_t rup_sz(size_t v, size_t a) { return (v + a - 1) / a * a; }
int rup_i(int v, int a) { return (v + a - 1) / a * a; }

// A bump planner over the caller's workspace: the same walk sizes it (base == nullptr) and
// hands out the pieces.
struct Plan {
    char* base;
    size_t used = 0;
    explicit Plan(void* b) : base(static_cast<char*>(b)) {}
    void* take(size_t bytes) {
        void* p = base ? base + used : nullptr;
        used += rup_sz(bytes, kAlign);
        return p;
    }
};

// The network's buffer geometry (copenerf.fields.SDFNetwork.layout / SDFLayout).
struct NetShape {
    int L8, E, KE, HL, sk;
    bool bf, x6, img, fuse_head, fused;
};

int net_shape(const cn_sdf_net* n, NetShape* s) {
    CN_REQUIRE(n, CN_ERR_ARG, "cn_sdf_net: null");
    CN_REQUIRE(n->n_lin >= 2 && n->n_lin <= CN_SDF_MAX_LIN, CN_ERR_SHAPE, "cn_sdf_net: n_lin %d (2 .. %d)", n->n_lin,
               CN_SDF_MAX_LIN);
    CN_REQUIRE(n->mfma_dtype >= CN_MFMA_F32 && n->mfma_dtype <= CN_MFMA_F32_BF16X6, CN_ERR_ARG,
               "cn_sdf_net: mfma_dtype %d", n->mfma_dtype);
    CN_REQUIRE(n->multires >= 0 && n->multires <= 12, CN_ERR_SHAPE, "cn_sdf_net: multires %d", n->multires);
    const int L8 = n->n_lin - 1;
    s->L8 = L8;
    s->E = 4 * (1 + 2 * n->multires);
    s->KE = rup_i(s->E, 64);
    s->sk = n->skip;
    CN_REQUIRE(s->sk == -1 || (s->sk >= 1 && s->sk <= L8), CN_ERR_SHAPE, "cn_sdf_net: skip %d", s->sk);
    int hl = 0;
    for (int l = 0; l <= L8; ++l) {
        CN_REQUIRE(n->in_dim[l] >= 1 && n->out_dim[l] >= 1, CN_ERR_SHAPE, "cn_sdf_net: layer %d dims", l);
        if (l >= 1) hl = n->in_dim[l] > hl ? n->in_dim[l] : hl;
        if (l < L8) hl = n->out_dim[l] > hl ? n->out_dim[l] : hl;
    }
    s->HL = rup_i(hl, 128);
    CN_REQUIRE(n->in_dim[0] == s->E, CN_ERR_SHAPE, "cn_sdf_net: lin0 takes %d inputs, the encoding has %d",
               n->in_dim[0], s->E);
    for (int l = 1; l <= L8; ++l) {
        const int want = n->out_dim[l - 1] + (l == s->sk ? s->E : 0);
        CN_REQUIRE(n->in_dim[l] == want, CN_ERR_SHAPE, "cn_sdf_net: lin%d takes %d inputs, expected %d", l,
                   n->in_dim[l], want);
    }
    s->x6 = n->mfma_dtype == CN_MFMA_F32_BF16X6;
    s->bf = n->mfma_dtype == CN_MFMA_BF16;
    const int kq = s->bf ? 64 : 32;
    for (int l = 0; l < L8; ++l) {
        const int kp = l == 0 ? s->KE : rup_i(n->in_dim[l], kq);
        CN_REQUIRE(n->W[l] && n->bias[l], CN_ERR_ARG, "cn_sdf_net: layer %d weights / bias null", l);
        CN_REQUIRE(((uintptr_t)n->bias[l] & 15) == 0 && ((uintptr_t)n->W[l] & 15) == 0, CN_ERR_ALIGN,
                   "cn_sdf_net: layer %d weights / bias not 16-byte aligned", l);
        CN_REQUIRE(n->w_rows[l] >= rup_i(n->out_dim[l], 128) && n->w_cols[l] >= kp && n->w_cols[l] % kq == 0,
                   CN_ERR_SHAPE, "cn_sdf_net: layer %d image [%d][%d] too small for %d x %d", l, n->w_rows[l],
                   n->w_cols[l], n->out_dim[l], kp);
    }
    CN_REQUIRE(n->head_w && n->head_b, CN_ERR_ARG, "cn_sdf_net: head null");
    CN_REQUIRE(((uintptr_t)n->head_w & 15) == 0, CN_ERR_ALIGN, "cn_sdf_net: head_w not 16-byte aligned");
    // bf16 operand images for the hidden activations (fields._img_mode)
    s->img = s->bf && s->HL % 256 == 0;
    // the sdf head in the last hidden layer's epilogue (fields._fuse_head)
    {
        const int N = n->out_dim[L8 - 1];
        const bool shape_ok = n->in_dim[L8] == N && N % 4 == 0 && L8 != s->sk && L8 - 1 != 0;
        s->fuse_head = shape_ok && (N <= 128 ||
                                    (s->x6 && N <= 256 && n->w_rows[L8 - 1] >= 256 &&
                                     rup_i(n->in_dim[L8 - 1], 32) % 64 == 0) ||
                                    (s->bf && N <= 256 && n->w_rows[L8 - 1] >= 256));
    }
    // cn_sdf_mlp's shape (fields._fused_query_ok)
    bool f = !(n->flags & CN_SDF_LAYERED) && s->img && n->n_lin == 9 && s->HL == 256 && s->KE == 64 &&
             s->sk >= 2 && s->sk <= 7;
    if (f) f = s->E + n->out_dim[s->sk - 1] == 256 && n->in_dim[8] == 256;
    for (int l = 0; f && l < 8; ++l)
        f = (l == s->sk - 1 || n->out_dim[l] == 256) && n->w_rows[l] == 256;
    s->fused = f;
    return CN_OK;
}

int sdf_query_plan(const cn_sdf_net* n, const NetShape& s, int M, const float* x, int64_t ldx, float* sdf,
                   const int32_t* idx, Plan& ws, hipStream_t st, bool run) {
    const float kSqrt2 = (float)std::sqrt(2.0);
    if (s.fused) {
        // cn_sdf_embed's bf16 images (lin0's input; the skip concat's tail / sqrt 2), then one cn_sdf_mlp
        void* u0b = ws.take((size_t)M * 64 * 2);
        void* tail = ws.take((size_t)M * 64 * 2);
        if (!run) return CN_OK;
        int rc = cn_sdf_embed(M, x, ldx, n->multires, n->scale, 64, u0b, 64, tail, 64, kSqrt2, 3, st);
        if (rc) return rc;
        cn_sdf_mlp_desc d{};
        d.u0 = u0b;
        d.tail = tail;
        d.ld_u0 = 64;
        d.ld_t = 64;
        d.M = M;
        d.n_layers = 8;
        d.hidden = 256;
        d.kpad0 = 64;
        d.multires = n->multires;
        d.skip_layer = s.sk - 1;
        for (int l = 0; l < 8; ++l) {
            d.W[l] = n->W[l];
            d.ldw[l] = n->w_cols[l];
            d.bias[l] = n->bias[l];
        }
        d.head_w = n->head_w;
        d.head_b = n->head_b;
        d.sdf = sdf;
        d.idx = idx;
        d.skip_div = kSqrt2;
        d.beta = n->beta;
        d.threshold = n->threshold;
        return cn_sdf_mlp(&d, st);
    }
    // layer by layer (fields.sdf_forward): U0 fp32 [M][KE]; the skip layer's input Usk (bf16 image in the
    // image mode, its tail written by the embedding); two ping-pong activation buffers
    const int L8 = s.L8, HL = s.HL, sk = s.sk;
    const bool usk_b = s.img && sk >= 1 && sk < L8;
    const size_t pp_elem = (s.img && s.fuse_head) ? 2 : 4;  // only bf16 images (and no stored U_8) then
    float* U0 = static_cast<float*>(ws.take((size_t)M * s.KE * 4));
    char* Usk = sk >= 0 ? static_cast<char*>(ws.take((size_t)M * HL * (usk_b ? 2 : 4))) : nullptr;
    char* pp[2] = {static_cast<char*>(ws.take((size_t)M * HL * pp_elem)),
                   static_cast<char*>(ws.take((size_t)M * HL * pp_elem))};
    if (!run) return CN_OK;
    void* e_view = nullptr;
    if (sk >= 0) e_view = Usk + (size_t)n->out_dim[sk - 1] * (usk_b ? 2 : 4);
    int rc = cn_sdf_embed(M, x, ldx, n->multires, n->scale, s.KE, U0, s.KE, e_view, e_view ? HL : 0, kSqrt2,
                          usk_b ? 1 : 0, st);
    if (rc) return rc;
    const void* A = U0;
    int64_t lda = s.KE;
    bool a_b = false;
    const void* U8 = nullptr;
    for (int l = 0; l < L8; ++l) {
        const bool into = (l + 1) == sk;
        int K = l == 0 ? s.KE : rup_i(n->in_dim[l], 32);
        if (s.bf) K = rup_i(K, 64);
        cn_linear_desc d{};
        d.A = A;
        d.lda = lda;
        d.a_bf16 = a_b ? 1 : 0;
        d.B = static_cast<const float*>(n->W[l]);
        d.ldb = s.x6 ? n->w_rows[l] : n->w_cols[l];
        d.bias = n->bias[l];
        d.M = M;
        d.N = n->out_dim[l];
        d.K = d.K1 = K;
        d.nsplit = d.N;
        d.adiv = 1.0f;
        d.odiv = 1.0f;
        d.beta = n->beta;
        d.threshold = n->threshold;
        d.mfma_dtype = n->mfma_dtype;
        d.flags = l & 1;  // consecutive launches walk the rows in opposite directions (results do not depend on it)
        void* out = nullptr;
        void* outb = nullptr;
        if (l == L8 - 1 && s.fuse_head) {
            d.epilogue = CN_EPI_SOFTPLUS_HEAD;
            d.nzero = HL;
            d.head_w = n->head_w;
            d.head_b = n->head_b;
            d.head_out = sdf;
            d.head_idx = idx;
        } else {
            d.epilogue = CN_EPI_SOFTPLUS;
            d.nzero = into ? n->out_dim[l] : HL;
            if (into) d.odiv = kSqrt2;
            char* dst = into ? Usk : pp[l & 1];
            if (s.img && l + 1 < L8) {  // the next layer's operand image, the activation's only copy
                outb = dst;
                d.out0_b = outb;
                d.ld_out0_b = HL;
            } else {
                out = dst;
                d.out0 = static_cast<float*>(out);
                d.ld_out0 = HL;
            }
        }
        d.tile = (d.N <= 64 && d.nzero <= 64) ? 1 : 0;
        rc = cn_linear(&d, st);
        if (rc) return rc;
        A = out ? out : outb;
        a_b = outb != nullptr;
        lda = HL;
        if (l == L8 - 1) U8 = out;
    }
    if (!s.fuse_head)
        return cn_row_head(M, n->in_dim[L8], static_cast<const float*>(U8), HL, n->head_w, n->in_dim[L8],
                           n->head_b, 1, 0, sdf, 1, idx, st);
    return CN_OK;
}

int query_check(const cn_sdf_net* n, int32_t M, const float* x, int64_t ldx, float* sdf) {
    CN_REQUIRE(M >= 0, CN_ERR_SHAPE, "cn_sdf_query: M = %d", M);
    CN_REQUIRE(M == 0 || (x && sdf), CN_ERR_ARG, "cn_sdf_query: null x / sdf");
    CN_REQUIRE(ldx >= 4, CN_ERR_SHAPE, "cn_sdf_query: ldx %lld < 4", (long long)ldx);
    (void)n;
    return CN_OK;
}

// The sampler's buffers: two ping-pong z / sdf rows of the final width, the points of the widest
// query, the new samples and their scatter targets, then the query's own workspace (reused by
// every round: the stream orders them).
struct SamplePlan {
    float *z[2], *sdf[2], *pts, *z_new;
    int32_t* dst;
    int k, width, qmax;
};

int sample_plan(const cn_sample_desc* d, const NetShape& s, Plan& ws, SamplePlan* p) {
    const int R = d->R, ns = d->n_samples;
    p->k = d->n_importance > 0 ? d->n_importance / d->up_sample_steps : 0;
    p->width = ns + d->up_sample_steps * p->k;
    p->qmax = ns > p->k ? ns : p->k;
    const size_t rows = (size_t)R * p->width;
    for (int i = 0; i < 2; ++i) {
        p->z[i] = static_cast<float*>(ws.take(rows * 4));
        p->sdf[i] = static_cast<float*>(ws.take(rows * 4));
    }
    p->pts = static_cast<float*>(ws.take((size_t)R * p->qmax * 16));
    p->z_new = static_cast<float*>(ws.take((size_t)R * (p->k > 0 ? p->k : 1) * 4));
    p->dst = static_cast<int32_t*>(ws.take((size_t)R * (p->k > 0 ? p->k : 1) * 4));
    (void)s;
    return CN_OK;
}

int sample_check(const cn_sample_desc* d) {
    CN_REQUIRE(d, CN_ERR_ARG, "cn_sample: null descriptor");
    CN_REQUIRE(d->R >= 0 && d->n_samples >= 1 && d->n_importance >= 0, CN_ERR_SHAPE,
               "cn_sample: R %d n_samples %d n_importance %d", d->R, d->n_samples, d->n_importance);
    CN_REQUIRE(d->n_importance == 0 || (d->up_sample_steps >= 1 && d->n_importance >= d->up_sample_steps),
               CN_ERR_SHAPE, "cn_sample: n_importance %d over %d up-sample steps", d->n_importance, d->up_sample_steps);
    CN_REQUIRE(d->near && d->far && d->z, CN_ERR_ARG, "cn_sample: null near / far / z");
    CN_REQUIRE(d->n_importance == 0 || (d->rays_o && d->rays_d && d->time_step && d->net), CN_ERR_ARG,
               "cn_sample: null rays / time_step / net");
    return CN_OK;
}

}  // namespace

extern "C" size_t cn_sdf_query_workspace_bytes(const cn_sdf_net* net, int32_t M) {
    NetShape s;
    if (M < 0 || net_shape(net, &s) != CN_OK) return 0;
    Plan ws(nullptr);
    sdf_query_plan(net, s, M, nullptr, 4, nullptr, nullptr, ws, nullptr, false);
    return ws.used;
}

extern "C" int cn_sdf_query(const cn_sdf_net* net, int32_t M, const float* x, int64_t ldx, float* sdf,
                            const int32_t* idx, void* workspace, int64_t workspace_bytes, cn_stream_t stream) {
    NetShape s;
    int rc = net_shape(net, &s);
    if (rc) return rc;
    if ((rc = query_check(net, M, x, ldx, sdf))) return rc;
    if (M == 0) return CN_OK;
    const size_t need = cn_sdf_query_workspace_bytes(net, M);
    CN_REQUIRE(workspace && workspace_bytes >= 0 && (size_t)workspace_bytes >= need, CN_ERR_SHAPE,
               "cn_sdf_query: workspace %lld bytes, %zu needed", (long long)workspace_bytes, need);
    CN_REQUIRE(((uintptr_t)workspace & (kAlign - 1)) == 0, CN_ERR_ALIGN, "cn_sdf_query: workspace not 256-byte aligned");
    Plan ws(workspace);
    return sdf_query_plan(net, s, M, x, ldx, sdf, idx, ws, (hipStream_t)stream, true);
}

extern "C" size_t cn_sample_workspace_bytes(const cn_sample_desc* d) {
    if (sample_check(d) != CN_OK) return 0;
    if (d->n_importance == 0) return 0;
    NetShape s;
    if (net_shape(d->net, &s) != CN_OK) return 0;
    Plan ws(nullptr);
    SamplePlan p;
    sample_plan(d, s, ws, &p);
    return ws.used + cn_sdf_query_workspace_bytes(d->net, d->R * p.qmax);
}

extern "C" int cn_sample(const cn_sample_desc* d, void* workspace, int64_t workspace_bytes, cn_stream_t stream) {
    int rc = sample_check(d);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int R = d->R, ns = d->n_samples;
    if (d->n_importance == 0) return cn_coarse_z(R, ns, d->near, d->far, d->t_rand, d->z, stream);
    NetShape s;
    if ((rc = net_shape(d->net, &s))) return rc;
    if (R == 0) return CN_OK;
    const size_t need = cn_sample_workspace_bytes(d);
    CN_REQUIRE(workspace && workspace_bytes >= 0 && (size_t)workspace_bytes >= need, CN_ERR_SHAPE,
               "cn_sample: workspace %lld bytes, %zu needed", (long long)workspace_bytes, need);
    CN_REQUIRE(((uintptr_t)workspace & (kAlign - 1)) == 0, CN_ERR_ALIGN, "cn_sample: workspace not 256-byte aligned");
    CN_REQUIRE((int64_t)R * (ns > d->n_importance ? ns : d->n_importance) < ((int64_t)1 << 31) &&
                   (int64_t)R * (ns + d->n_importance) < ((int64_t)1 << 31),
               CN_ERR_SHAPE, "cn_sample: R = %d too large", R);
    Plan ws(workspace);
    SamplePlan p;
    sample_plan(d, s, ws, &p);
    char* qws = ws.base + ws.used;
    const int64_t qbytes = workspace_bytes - (int64_t)ws.used;
    // coarse samples and their SDF (neus_renderer.py:466-498)
    float* z = p.z[0];
    float* sdf = p.sdf[0];
    if ((rc = cn_coarse_z(R, ns, d->near, d->far, d->t_rand, z, stream))) return rc;
    if ((rc = cn_points(R, ns, d->rays_o, d->rays_d, z, d->time_step, 0, nullptr, nullptr, 0, p.pts, stream)))
        return rc;
    if ((rc = cn_sdf_query(d->net, R * ns, p.pts, 4, sdf, nullptr, qws, qbytes, stream))) return rc;
    // up_sample + cat_z_vals rounds (neus_renderer.py:500-520)
    int n = ns;
    for (int i = 0; i < d->up_sample_steps; ++i) {
        const bool last = i + 1 == d->up_sample_steps;
        float* z_out = last ? d->z : p.z[(i + 1) & 1];
        float* sdf_out = last ? nullptr : p.sdf[(i + 1) & 1];
        const float inv_s = 64.0f * (float)(1 << i);
        if ((rc = cn_up_sample_merge(R, n, p.k, inv_s, z, sdf, z_out, p.z_new, sdf_out, last ? nullptr : p.dst, stream)))
            return rc;
        if (!last) {
            if ((rc = cn_points(R, p.k, d->rays_o, d->rays_d, p.z_new, d->time_step, 0, nullptr, nullptr, 0, p.pts,
                                stream)))
                return rc;
            if ((rc = cn_sdf_query(d->net, R * p.k, p.pts, 4, sdf_out, p.dst, qws, qbytes, stream))) return rc;
        }
        z = z_out;
        sdf = sdf_out;
        n += p.k;
    }
    (void)st;
    return CN_OK;
}
