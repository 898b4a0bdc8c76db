// cn_render.hip — sampling along rays and alpha compositing (gfx950).
//
// One wavefront (64 lanes) per ray.  A ray's S <= 256 samples are held as
// contiguous chunks of P = ceil(S/64) samples per lane, so the transmittance
// cumprod, the pdf cumsum and the backward suffix sums are a per-lane chunk
// scan plus one 6-step wavefront scan (__shfl_up).  The scans accumulate in
// double and round each output to fp32: that is what torch's CPU cumprod /
// cumsum do (acc_type<float, /*is_cuda=*/false> = double), so the sampled
// z-values of the oracle are reproduced far more often than with fp32 scans.
#include "cn_common.h"

namespace cn {

constexpr int kMaxPerLane = 4;  // S <= 256 samples per ray
constexpr int kRaysPerBlock = 4;

template <typename T>
__device__ __forceinline__ T wave_incl_scan_add(T x, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// inclusive suffix sum over lanes: x_lane + x_{lane+1} + ... + x_63
__device__ __forceinline__ double wave_incl_suffix_add(double x, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_down(x, off, 64);
        if (lane + off < 64) x += y;
    }
    return x;
}

__device__ __forceinline__ double wave_incl_scan_mul(double x, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_up(x, off, 64);
        if (lane >= off) x *= y;
    }
    return x;
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// torch.linspace(0, 1, n) on CPU (scalar form of RangeFactoriesKernel.cpp).
__device__ __forceinline__ float linspace01(int i, int n) {
    if (n == 1) return 0.0f;
    const float step = (1.0f - 0.0f) / (float)(n - 1);
    const int half = n / 2;
    return i < half ? 0.0f + step * (float)i : 1.0f - step * (float)(n - i - 1);
}

__global__ void coarse_z_kernel(int R, int n, const float* __restrict__ near, const float* __restrict__ far,
                                const float* __restrict__ t_rand, float* z) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)R * n) return;
    const int r = idx / n, i = idx % n;
    const float nr = near[r], fr = far[r];
    auto zl = [&](int j) { const float l = linspace01(j, n); return nr * (1.0f - l) + fr * l; };
    const float zi = zl(i);
    if (!t_rand) {
        z[idx] = zi;
        return;
    }
    // neus_renderer.py:478-483: mids / upper / lower, z = lower + (upper - lower) * t
    const float upper = i < n - 1 ? 0.5f * (zl(i + 1) + zi) : zi;
    const float lower = i > 0 ? 0.5f * (zi + zl(i - 1)) : zi;
    z[idx] = lower + (upper - lower) * t_rand[idx];
}

// Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11; the Random123
// constants): ten rounds of two 32x32 -> 64-bit multiplies, the key bumped by the Weyl constants between rounds.
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = (uint32_t)p1;
        c[2] = n2;
        c[3] = (uint32_t)p0;
    }
}

// out[i] = the 24 high bits of word i % 4 of Philox4x32-10(counter (i / 4, offset), key seed) x 2^-24, in [0, 1);
// seed and offset are read on the device (so = [seed, offset]: a captured launch replays with the current values)
__global__ void __launch_bounds__(256) uniform_philox_kernel(int64_t n, const uint64_t* __restrict__ so,
                                                             float* __restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g * 4 >= n) return;
    const uint64_t seed = so[0], off = so[1];
    uint32_t c[4] = {(uint32_t)g, (uint32_t)((uint64_t)g >> 32), (uint32_t)off, (uint32_t)(off >> 32)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    for (int k = 0; k < 4 && g * 4 + k < n; ++k) out[g * 4 + k] = (float)(c[k] >> 8) * (1.0f / 16777216.0f);
}

__global__ void points_kernel(int R, int n, const float* __restrict__ o, const float* __restrict__ d,
                              const float* __restrict__ z, const float* __restrict__ tptr, int mid,
                              const float* __restrict__ near, const float* __restrict__ far, int n_coarse,
                              float* pts) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)R * n) return;
    const int r = idx / n, i = idx % n;
    float zz = z[idx];
    if (mid) {
        const float dist = i < n - 1 ? z[idx + 1] - zz : (far[0] - near[0]) / (float)n_coarse;
        zz = zz + dist * 0.5f;
    }
    floatx4 p;
    for (int c = 0; c < 3; ++c) p[c] = o[3 * r + c] + d[3 * r + c] * zz;
    p[3] = tptr[0];
    *reinterpret_cast<floatx4*>(pts + 4 * idx) = p;
}

// Backward of points_kernel: one wavefront per ray, lanes stride the samples.
__global__ void __launch_bounds__(256) points_bwd_kernel(int R, int n, const float* __restrict__ z, int mid,
                                                         const float* __restrict__ near, const float* __restrict__ far,
                                                         int n_coarse, const float* __restrict__ dP, int64_t ld_p,
                                                         float* drays_o, float* drays_d) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * kRaysPerBlock + (threadIdx.x >> 6);
    if (r >= R) return;
    double so[3] = {0.0, 0.0, 0.0}, sd[3] = {0.0, 0.0, 0.0};
    for (int i = lane; i < n; i += 64) {
        const int64_t idx = (int64_t)r * n + i;
        float zz = z[idx];
        if (mid) {
            const float dist = i < n - 1 ? z[idx + 1] - zz : (far[0] - near[0]) / (float)n_coarse;
            zz = zz + dist * 0.5f;
        }
        for (int c = 0; c < 3; ++c) {
            const float g = dP[idx * ld_p + c];
            so[c] += (double)g;
            sd[c] += (double)(g * zz);
        }
    }
    for (int c = 0; c < 3; ++c) {
        const double a = wave_sum(so[c]), b = wave_sum(sd[c]);
        if (lane == 0) {
            if (drays_o) drays_o[3 * r + c] = (float)a;
            if (drays_d) drays_d[3 * r + c] = (float)b;
        }
    }
}

// One NeuS up-sampling round (up_sample + sample_pdf(det) + cat_z_vals).
__global__ void __launch_bounds__(256) up_sample_merge_kernel(int R, int n, int n_imp, float inv_s,
                                                              const float* __restrict__ z,
                                                              const float* __restrict__ sdf, float* z_out,
                                                              float* z_new, float* sdf_out, int* new_dst) {
    constexpr int NMAX = 256;
    __shared__ float s_z[kRaysPerBlock][NMAX];
    __shared__ float s_s[kRaysPerBlock][NMAX];
    __shared__ float s_cdf[kRaysPerBlock][NMAX];
    __shared__ float s_new[kRaysPerBlock][64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int r = blockIdx.x * kRaysPerBlock + wv;
    const bool active = r < R;
    float* zs = s_z[wv];
    float* ss = s_s[wv];
    float* cs = s_cdf[wv];
    float* zn = s_new[wv];

    if (active) {
        for (int i = lane; i < n; i += 64) {
            zs[i] = z[(int64_t)r * n + i];
            ss[i] = sdf[(int64_t)r * n + i];
        }
    }
    __syncthreads();

    const int nI = n - 1;  // intervals
    const int P = cdiv(nI, 64);
    float alpha[kMaxPerLane], cp[kMaxPerLane];
    double lprod = 1.0;
#pragma unroll
    for (int p = 0; p < kMaxPerLane; ++p) {
        alpha[p] = 0.0f;
        cp[p] = 1.0f;
        const int i = lane * P + p;
        if (!active || p >= P || i >= nI) continue;
        const float z0 = zs[i], z1 = zs[i + 1], s0 = ss[i], s1 = ss[i + 1];
        const float mid_sdf = (s0 + s1) * 0.5f;
        const float cv = (s1 - s0) / (z1 - z0 + 1e-5f);
        const float pcv = i == 0 ? 0.0f : (s0 - ss[i - 1]) / (z0 - zs[i - 1] + 1e-5f);
        float c = pcv < cv ? pcv : cv;  // torch.min over the stacked pair
        c = c < -1e3f ? -1e3f : (c > 0.0f ? 0.0f : c);
        const float dist = z1 - z0;
        const float prev_e = mid_sdf - c * dist * 0.5f;
        const float next_e = mid_sdf + c * dist * 0.5f;
        const float prev_c = sigmoidf_ref(prev_e * inv_s);
        const float next_c = sigmoidf_ref(next_e * inv_s);
        alpha[p] = (prev_c - next_c + 1e-5f) / (prev_c + 1e-5f);
        cp[p] = 1.0f - alpha[p] + 1e-7f;
        lprod *= (double)cp[p];
    }
    // exclusive product scan -> T_i, weights = alpha * T
    const double incl = wave_incl_scan_mul(lprod, lane);
    double excl = __shfl_up(incl, 1, 64);
    if (lane == 0) excl = 1.0;
    float wts[kMaxPerLane];
    double lsum = 0.0;
    {
        double run = excl;
#pragma unroll
        for (int p = 0; p < kMaxPerLane; ++p) {
            const int i = lane * P + p;
            wts[p] = 0.0f;
            if (!active || p >= P || i >= nI) continue;
            const float T = (float)run;
            run *= (double)cp[p];
            wts[p] = alpha[p] * T + 1e-5f;  // sample_pdf: weights + 1e-5
            lsum += (double)wts[p];
        }
    }
    const float total = (float)wave_sum(lsum);
    // cdf = cumsum(pdf), pdf = w / total; cdf_full = [0, cdf]
    float pdf[kMaxPerLane];
    double lcs = 0.0;
#pragma unroll
    for (int p = 0; p < kMaxPerLane; ++p) {
        const int i = lane * P + p;
        pdf[p] = 0.0f;
        if (!active || p >= P || i >= nI) continue;
        pdf[p] = wts[p] / total;
        lcs += (double)pdf[p];
    }
    const double cincl = wave_incl_scan_add(lcs, lane);
    double cexcl = __shfl_up(cincl, 1, 64);
    if (lane == 0) cexcl = 0.0;
    if (active) {
        double run = cexcl;
#pragma unroll
        for (int p = 0; p < kMaxPerLane; ++p) {
            const int i = lane * P + p;
            if (p >= P || i >= nI) continue;
            run += (double)pdf[p];
            cs[i + 1] = (float)run;
        }
        if (lane == 0) cs[0] = 0.0f;
    }
    __syncthreads();

    // inverse CDF at u_k = linspace(0.5/n_imp, 1 - 0.5/n_imp, n_imp)
    if (active && lane < n_imp) {
        const float u0 = 0.5f / (float)n_imp, u1 = 1.0f - 0.5f / (float)n_imp;
        const float step = n_imp > 1 ? (u1 - u0) / (float)(n_imp - 1) : 0.0f;
        const float u = lane < n_imp / 2 ? u0 + step * (float)lane : u1 - step * (float)(n_imp - lane - 1);
        // searchsorted(cdf, u, right=True) = #{j : cdf[j] <= u}
        int lo = 0, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cs[mid] <= u) lo = mid + 1;
            else hi = mid;
        }
        const int below = lo - 1 > 0 ? lo - 1 : 0;
        const int above = lo < n - 1 ? lo : n - 1;
        const float c0 = cs[below], c1 = cs[above];
        float denom = c1 - c0;
        denom = denom < 1e-5f ? 1.0f : denom;
        const float t = (u - c0) / denom;
        const float b0 = zs[below], b1 = zs[above];
        zn[lane] = b0 + t * (b1 - b0);
    }
    __syncthreads();

    if (!active) return;
    const int nt = n + n_imp;
    // merge (stable: old before new on ties; new samples need not be sorted)
    for (int i = lane; i < n; i += 64) {
        const float zi = zs[i];
        int cnt = 0;
        for (int k = 0; k < n_imp; ++k) cnt += zn[k] < zi ? 1 : 0;
        const int pos = i + cnt;
        z_out[(int64_t)r * nt + pos] = zi;
        if (sdf_out) sdf_out[(int64_t)r * nt + pos] = ss[i];
    }
    if (lane < n_imp) {
        const float zk = zn[lane];
        int lo = 0, hi = n;  // upper_bound in the sorted old list
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (zs[mid] <= zk) lo = mid + 1;
            else hi = mid;
        }
        int cnt = lo;
        for (int k = 0; k < n_imp; ++k) {
            const float zq = zn[k];
            cnt += (zq < zk || (zq == zk && k < lane)) ? 1 : 0;
        }
        z_out[(int64_t)r * nt + cnt] = zk;
        z_new[(int64_t)r * n_imp + lane] = zk;
        if (new_dst) new_dst[(int64_t)r * n_imp + lane] = r * nt + cnt;
    }
}

// ---------------------------------------------------------------------------
// Compositing (render_core, neus_renderer.py:337-420).
struct SampleState {
    float z, dist, sdf, n0, n1, n2, tc, ic, en, ep, pc, nc, q, alpha, cp;
};

__device__ __forceinline__ void composite_sample(SampleState& s, const float* d, float inv_s, float car) {
    s.tc = d[0] * s.n0 + d[1] * s.n1 + d[2] * s.n2;
    const float ra = -s.tc * 0.5f + 0.5f;
    const float rb = -s.tc;
    s.ic = -((ra > 0.0f ? ra : 0.0f) * (1.0f - car) + (rb > 0.0f ? rb : 0.0f) * car);
    const float h = s.ic * s.dist * 0.5f;
    s.en = s.sdf + h;
    s.ep = s.sdf - h;
    s.pc = sigmoidf_ref(s.ep * inv_s);
    s.nc = sigmoidf_ref(s.en * inv_s);
    const float pp = s.pc - s.nc;
    s.q = (pp + 1e-5f) / (s.pc + 1e-5f);
    s.alpha = s.q < 0.0f ? 0.0f : (s.q > 1.0f ? 1.0f : s.q);
    s.cp = 1.0f - s.alpha + 1e-7f;
}

__device__ __forceinline__ void load_sample(SampleState& s, int r, int i, int S, const float* z, const float* sdf,
                                            const float* G, int64_t ld_g, float sample_dist) {
    const int64_t m = (int64_t)r * S + i;
    s.z = z[m];
    s.dist = i < S - 1 ? z[m + 1] - s.z : sample_dist;
    s.sdf = sdf[m];
    s.n0 = G[m * ld_g];
    s.n1 = G[m * ld_g + 1];
    s.n2 = G[m * ld_g + 2];
}

__global__ void __launch_bounds__(256) composite_fwd_kernel(int R, int S, const float* __restrict__ z,
                                                            const float* __restrict__ sdf, const float* __restrict__ G,
                                                            int64_t ld_g, const float* __restrict__ rgb,
                                                            const float* __restrict__ rays_d,
                                                            const float* __restrict__ inv_s_p,
                                                            const float* __restrict__ near,
                                                            const float* __restrict__ far, int n_coarse,
                                                            const float* __restrict__ car_p,
                                                            float* color, float* depth, float* weights, float* cdf) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * kRaysPerBlock + (threadIdx.x >> 6);
    if (r >= R) return;
    const float inv_s = inv_s_p[0];
    const float car = car_p[0];
    const float sample_dist = (far[0] - near[0]) / (float)n_coarse;
    const float d[3] = {rays_d[3 * r], rays_d[3 * r + 1], rays_d[3 * r + 2]};
    const int P = cdiv(S, 64);
    SampleState st[kMaxPerLane];
    double lprod = 1.0;
#pragma unroll
    for (int p = 0; p < kMaxPerLane; ++p) {
        const int i = lane * P + p;
        if (p >= P || i >= S) continue;
        load_sample(st[p], r, i, S, z, sdf, G, ld_g, sample_dist);
        composite_sample(st[p], d, inv_s, car);
        lprod *= (double)st[p].cp;
    }
    const double incl = wave_incl_scan_mul(lprod, lane);
    double run = __shfl_up(incl, 1, 64);
    if (lane == 0) run = 1.0;
    double c0 = 0.0, c1 = 0.0, c2 = 0.0, dz = 0.0;
#pragma unroll
    for (int p = 0; p < kMaxPerLane; ++p) {
        const int i = lane * P + p;
        if (p >= P || i >= S) continue;
        const float T = (float)run;
        run *= (double)st[p].cp;
        const float w = st[p].alpha * T;
        const int64_t m = (int64_t)r * S + i;
        weights[m] = w;
        if (cdf) cdf[m] = st[p].pc;
        c0 += (double)(rgb[3 * m] * w);
        c1 += (double)(rgb[3 * m + 1] * w);
        c2 += (double)(rgb[3 * m + 2] * w);
        dz += (double)(st[p].z * w);
    }
    c0 = wave_sum(c0);
    c1 = wave_sum(c1);
    c2 = wave_sum(c2);
    dz = wave_sum(dz);
    if (lane == 0) {
        color[3 * r] = (float)c0;
        color[3 * r + 1] = (float)c1;
        color[3 * r + 2] = (float)c2;
        depth[r] = (float)dz;
    }
}

__global__ void __launch_bounds__(256) composite_bwd_kernel(
    int R, int S, const float* __restrict__ z, const float* __restrict__ sdf, const float* __restrict__ G, int64_t ld_g,
    const float* __restrict__ rgb, const float* __restrict__ rays_d, const float* __restrict__ inv_s_p,
    const float* __restrict__ near, const float* __restrict__ far, int n_coarse, const float* __restrict__ car_p,
    const float* __restrict__ dcolor, const float* __restrict__ ddepth, const float* __restrict__ dweights,
    const float* __restrict__ dcdf, float* dsdf, float* dG, float* drgb, float* dinv_part, float* drays_d) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * kRaysPerBlock + (threadIdx.x >> 6);
    if (r >= R) return;
    const float inv_s = inv_s_p[0];
    const float car = car_p[0];
    const float sample_dist = (far[0] - near[0]) / (float)n_coarse;
    const float d[3] = {rays_d[3 * r], rays_d[3 * r + 1], rays_d[3 * r + 2]};
    const float gc0 = dcolor ? dcolor[3 * r] : 0.0f;
    const float gc1 = dcolor ? dcolor[3 * r + 1] : 0.0f;
    const float gc2 = dcolor ? dcolor[3 * r + 2] : 0.0f;
    const float gd = ddepth ? ddepth[r] : 0.0f;
    const int P = cdiv(S, 64);
    SampleState st[kMaxPerLane];
    double lprod = 1.0;
#pragma unroll
    for (int p = 0; p < kMaxPerLane; ++p) {
        const int i = lane * P + p;
        if (p >= P || i >= S) continue;
        load_sample(st[p], r, i, S, z, sdf, G, ld_g, sample_dist);
        composite_sample(st[p], d, inv_s, car);
        lprod *= (double)st[p].cp;
    }
    const double incl = wave_incl_scan_mul(lprod, lane);
    double run = __shfl_up(incl, 1, 64);
    if (lane == 0) run = 1.0;
    float T[kMaxPerLane], w[kMaxPerLane], gw[kMaxPerLane], prodw[kMaxPerLane];
    double lsum = 0.0;
#pragma unroll
    for (int p = 0; p < kMaxPerLane; ++p) {
        const int i = lane * P + p;
        T[p] = w[p] = gw[p] = prodw[p] = 0.0f;
        if (p >= P || i >= S) continue;
        const int64_t m = (int64_t)r * S + i;
        T[p] = (float)run;
        run *= (double)st[p].cp;
        w[p] = st[p].alpha * T[p];
        // dL/dw: colour = sum_i w_i rgb_i, depth = sum_i z_i w_i, plus the weights output
        float g = gc0 * rgb[3 * m] + gc1 * rgb[3 * m + 1] + gc2 * rgb[3 * m + 2];
        g = g + gd * st[p].z;
        if (dweights) g = g + dweights[m];
        gw[p] = g;
        drgb[3 * m] = gc0 * w[p];
        drgb[3 * m + 1] = gc1 * w[p];
        drgb[3 * m + 2] = gc2 * w[p];
        // cumprod backward: w_k = P_k * dP_k, dP_k = gw_k * alpha_k
        prodw[p] = T[p] * (gw[p] * st[p].alpha);
        lsum += (double)prodw[p];
    }
    // reversed (suffix) cumsum of prodw: rc_j = sum_{k >= j} prodw_k; we need
    // rc_{i+1} (torch: reversed_cumsum(output * grad).div(input), double acc).
    const double sincl = wave_incl_suffix_add(lsum, lane);
    double after = __shfl_down(sincl, 1, 64);  // sum over lanes > lane
    if (lane == 63) after = 0.0;
    double dinv = 0.0;
    double dd0 = 0.0, dd1 = 0.0, dd2 = 0.0;  // d rays_d from true_cos
#pragma unroll
    for (int p = kMaxPerLane - 1; p >= 0; --p) {
        const int i = lane * P + p;
        if (p >= P || i >= S) continue;
        const float rc_next = (float)after;  // sum_{k > i}
        after += (double)prodw[p];
        const SampleState& s = st[p];
        float da = gw[p] * T[p];
        da = da - rc_next / s.cp;
        const float dq = (s.q >= 0.0f && s.q <= 1.0f) ? da : 0.0f;
        const float num = (s.pc - s.nc) + 1e-5f;
        const float den = s.pc + 1e-5f;
        const float dnum = dq / den;
        const float dden = -dq * ((num / den) / den);
        const int64_t m = (int64_t)r * S + i;
        float dpc = dnum + dden;
        if (dcdf) dpc = dpc + dcdf[m];
        const float dnc = -dnum;
        const float g1 = dpc * (1.0f - s.pc) * s.pc;
        const float g2 = dnc * (1.0f - s.nc) * s.nc;
        const float dep = g1 * inv_s;
        const float den_ = g2 * inv_s;
        dinv += (double)(g1 * s.ep) + (double)(g2 * s.en);
        dsdf[m] = den_ + dep;
        const float dic = (den_ * 0.5f) * s.dist + ((-dep) * 0.5f) * s.dist;
        const float dsum = -dic;
        const float dA = dsum * (1.0f - car);
        const float dB = dsum * car;
        const float ra = -s.tc * 0.5f + 0.5f;
        const float da1 = ra > 0.0f ? dA : 0.0f;
        const float dB1 = (-s.tc) > 0.0f ? dB : 0.0f;
        const float dtc = -(da1 * 0.5f) + (-dB1);
        dG[4 * m] = dtc * d[0];
        dG[4 * m + 1] = dtc * d[1];
        dG[4 * m + 2] = dtc * d[2];
        dG[4 * m + 3] = 0.0f;
        if (drays_d) {
            dd0 += (double)(dtc * G[m * ld_g]);
            dd1 += (double)(dtc * G[m * ld_g + 1]);
            dd2 += (double)(dtc * G[m * ld_g + 2]);
        }
    }
    dinv = wave_sum(dinv);
    if (lane == 0) dinv_part[r] = (float)dinv;
    if (drays_d) {
        dd0 = wave_sum(dd0);
        dd1 = wave_sum(dd1);
        dd2 = wave_sum(dd2);
        if (lane == 0) {
            drays_d[3 * r] = (float)dd0;
            drays_d[3 * r + 1] = (float)dd1;
            drays_d[3 * r + 2] = (float)dd2;
        }
    }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Keyed pseudo-random permutation of [0, n): a balanced 4-round Feistel network on 2*hb
// bits (2^(2 hb) >= n) with cycle walking (values >= n are permuted again; starting below
// n the walk returns below n, expected < 4 steps).  Round function: a 32-bit avalanche hash.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t feistel(uint32_t x, int hb, const uint32_t k[4]) {
    const uint32_t mask = (1u << hb) - 1u;
    uint32_t L = x >> hb, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t t = L ^ (mix32(R ^ k[r]) & mask);
        L = R;
        R = t;
    }
    return (L << hb) | R;
}

// One thread per patch: its corner and its ps x ps pixel ids.
__global__ void patch_indices_kernel(int h, int w, int ps, int np, int hb, const int* __restrict__ key, int64_t* idx) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const int wa = w - ps + 1;
    const uint32_t n = (uint32_t)(h - ps + 1) * (uint32_t)wa;
    const uint32_t k[4] = {(uint32_t)key[0], (uint32_t)key[1], (uint32_t)key[2], (uint32_t)key[3]};
    uint32_t x = (uint32_t)p;
    do {
        x = feistel(x, hb, k);
    } while (x >= n);
    const int row = (int)(x / (uint32_t)wa), col = (int)(x % (uint32_t)wa);
    int64_t* o = idx + (int64_t)p * ps * ps;
    for (int a = 0; a < ps; ++a)
        for (int b = 0; b < ps; ++b) o[a * ps + b] = (int64_t)(row + a) * w + col + b;
}

// 3x3 helpers for the Euler chain (row-major, sums in k order as a small torch matmul)
struct M3 {
    float m[9];
};
__device__ __forceinline__ M3 mul3(const M3& a, const M3& b) {
    M3 c;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c.m[3 * i + j] = a.m[3 * i] * b.m[j] + a.m[3 * i + 1] * b.m[3 + j] + a.m[3 * i + 2] * b.m[6 + j];
    return c;
}
__device__ __forceinline__ M3 mul3_tb(const M3& a, const M3& b) {  // a bᵀ
    M3 c;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c.m[3 * i + j] = a.m[3 * i] * b.m[3 * j] + a.m[3 * i + 1] * b.m[3 * j + 1] + a.m[3 * i + 2] * b.m[3 * j + 2];
    return c;
}
__device__ __forceinline__ M3 mul3_ta(const M3& a, const M3& b) {  // aᵀ b
    M3 c;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c.m[3 * i + j] = a.m[i] * b.m[j] + a.m[3 + i] * b.m[3 + j] + a.m[6 + i] * b.m[6 + j];
    return c;
}
__device__ __forceinline__ M3 rot_x(float a, bool d) {  // Rx(a) or dRx/da
    const float c = cosf(a), s = sinf(a);
    return d ? M3{{0, 0, 0, 0, -s, -c, 0, c, -s}} : M3{{1, 0, 0, 0, c, -s, 0, s, c}};
}
__device__ __forceinline__ M3 rot_y(float a, bool d) {
    const float c = cosf(a), s = sinf(a);
    return d ? M3{{-s, 0, c, 0, 0, 0, -c, 0, -s}} : M3{{c, 0, s, 0, 1, 0, -s, 0, c}};
}
__device__ __forceinline__ M3 rot_z(float a, bool d) {
    const float c = cosf(a), s = sinf(a);
    return d ? M3{{-s, -c, 0, c, -s, 0, 0, 0, 0}} : M3{{c, -s, 0, s, c, 0, 0, 0, 1}};
}

constexpr int kEulerMaxSteps = 64;

__global__ void euler_chain_kernel(int K, int n, const float* __restrict__ omega, int64_t ld_o,
                                   const float* __restrict__ vel, int64_t ld_v, const float* __restrict__ dt,
                                   float* P) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const float h = dt[k];
    M3 Q = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    float T[3] = {0.f, 0.f, 0.f};
    for (int s = 0; s < n; ++s) {
        const float* o = omega + (int64_t)(k * n + s) * ld_o;
        const float* v = vel + (int64_t)(k * n + s) * ld_v;
        const M3 A = mul3(mul3(rot_x(o[0] * h, false), rot_y(o[1] * h, false)), rot_z(o[2] * h, false));
        float Tn[3];
        for (int i = 0; i < 3; ++i) Tn[i] = (A.m[3 * i] * T[0] + A.m[3 * i + 1] * T[1] + A.m[3 * i + 2] * T[2]) + v[i] * h;
        for (int i = 0; i < 3; ++i) T[i] = Tn[i];
        Q = mul3(Q, A);
    }
    float* p = P + 16 * (int64_t)k;
    for (int i = 0; i < 3; ++i) {
        p[4 * i] = Q.m[3 * i];
        p[4 * i + 1] = Q.m[3 * i + 1];
        p[4 * i + 2] = Q.m[3 * i + 2];
        p[4 * i + 3] = T[i];
    }
    p[12] = 0.f;
    p[13] = 0.f;
    p[14] = 0.f;
    p[15] = 1.f;
}

// Reverse recurrence: with Q_{s+1} = Q_s A_s and T_{s+1} = A_s T_s + V_s,
//   gA_s = gT_{s+1} T_sᵀ + Q_sᵀ gQ_{s+1},  gV_s = gT_{s+1},  gT_s = A_sᵀ gT_{s+1},  gQ_s = gQ_{s+1} A_sᵀ,
// and the angles through A = Rx Ry Rz.
__global__ void euler_chain_bwd_kernel(int K, int n, const float* __restrict__ omega, int64_t ld_o,
                                       const float* __restrict__ vel, int64_t ld_v, const float* __restrict__ dt,
                                       const float* __restrict__ dP, float* domega, float* dvel) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const float h = dt[k];
    M3 Qs[kEulerMaxSteps];
    float Ts[kEulerMaxSteps][3];
    M3 Q = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    float T[3] = {0.f, 0.f, 0.f};
    for (int s = 0; s < n; ++s) {  // forward again, keeping Q_s, T_s
        Qs[s] = Q;
        for (int i = 0; i < 3; ++i) Ts[s][i] = T[i];
        const float* o = omega + (int64_t)(k * n + s) * ld_o;
        const float* v = vel + (int64_t)(k * n + s) * ld_v;
        const M3 A = mul3(mul3(rot_x(o[0] * h, false), rot_y(o[1] * h, false)), rot_z(o[2] * h, false));
        float Tn[3];
        for (int i = 0; i < 3; ++i) Tn[i] = (A.m[3 * i] * T[0] + A.m[3 * i + 1] * T[1] + A.m[3 * i + 2] * T[2]) + v[i] * h;
        for (int i = 0; i < 3; ++i) T[i] = Tn[i];
        Q = mul3(Q, A);
    }
    const float* g = dP + 16 * (int64_t)k;
    M3 gQ = {{g[0], g[1], g[2], g[4], g[5], g[6], g[8], g[9], g[10]}};
    float gT[3] = {g[3], g[7], g[11]};
    for (int s = n - 1; s >= 0; --s) {
        const float* o = omega + (int64_t)(k * n + s) * ld_o;
        const float a = o[0] * h, b = o[1] * h, c = o[2] * h;
        const M3 X = rot_x(a, false), Y = rot_y(b, false), Z = rot_z(c, false);
        const M3 A = mul3(mul3(X, Y), Z);
        M3 gA = mul3_ta(Qs[s], gQ);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) gA.m[3 * i + j] += gT[i] * Ts[s][j];
        float* dv = dvel + 3 * (int64_t)(k * n + s);
        for (int i = 0; i < 3; ++i) dv[i] = gT[i] * h;
        float gTn[3];
        for (int j = 0; j < 3; ++j) gTn[j] = A.m[j] * gT[0] + A.m[3 + j] * gT[1] + A.m[6 + j] * gT[2];
        for (int j = 0; j < 3; ++j) gT[j] = gTn[j];
        gQ = mul3_tb(gQ, A);
        const M3 dA[3] = {mul3(mul3(rot_x(a, true), Y), Z), mul3(mul3(X, rot_y(b, true)), Z),
                          mul3(mul3(X, Y), rot_z(c, true))};
        float* dw = domega + 3 * (int64_t)(k * n + s);
        for (int q = 0; q < 3; ++q) {
            float acc = 0.f;
            for (int e = 0; e < 9; ++e) acc += gA.m[e] * dA[q].m[e];
            dw[q] = acc * h;
        }
    }
}

}  // namespace cn

using namespace cn;

extern "C" int cn_euler_chain(int32_t K, int32_t n, const float* omega, int64_t ld_o, const float* vel, int64_t ld_v,
                              const float* dt, float* P, cn_stream_t stream) {
    CN_REQUIRE(omega && vel && dt && P, CN_ERR_ARG, "cn_euler_chain: null pointer");
    CN_REQUIRE(K >= 0 && n >= 1 && n <= kEulerMaxSteps && ld_o >= 3 && ld_v >= 3, CN_ERR_SHAPE,
               "cn_euler_chain: K=%d n=%d (n <= %d)", K, n, kEulerMaxSteps);
    if (K == 0) return CN_OK;
    euler_chain_kernel<<<(K + 63) / 64, 64, 0, (hipStream_t)stream>>>(K, n, omega, ld_o, vel, ld_v, dt, P);
    return check_launch("cn_euler_chain");
}

extern "C" int cn_euler_chain_bwd(int32_t K, int32_t n, const float* omega, int64_t ld_o, const float* vel,
                                  int64_t ld_v, const float* dt, const float* dP, float* domega, float* dvel,
                                  cn_stream_t stream) {
    CN_REQUIRE(omega && vel && dt && dP && domega && dvel, CN_ERR_ARG, "cn_euler_chain_bwd: null pointer");
    CN_REQUIRE(K >= 0 && n >= 1 && n <= kEulerMaxSteps && ld_o >= 3 && ld_v >= 3, CN_ERR_SHAPE,
               "cn_euler_chain_bwd: K=%d n=%d (n <= %d)", K, n, kEulerMaxSteps);
    if (K == 0) return CN_OK;
    euler_chain_bwd_kernel<<<(K + 63) / 64, 64, 0, (hipStream_t)stream>>>(K, n, omega, ld_o, vel, ld_v, dt, dP,
                                                                          domega, dvel);
    return check_launch("cn_euler_chain_bwd");
}

extern "C" int cn_patch_indices(int32_t h, int32_t w, int32_t ps, int32_t n_patches, const int32_t* key, int64_t* idx,
                                cn_stream_t stream) {
    CN_REQUIRE(key && idx, CN_ERR_ARG, "cn_patch_indices: null pointer");
    CN_REQUIRE(ps >= 1 && h >= ps && w >= ps && n_patches >= 0, CN_ERR_SHAPE, "cn_patch_indices: h=%d w=%d ps=%d",
               h, w, ps);
    const int64_t n = (int64_t)(h - ps + 1) * (w - ps + 1);
    CN_REQUIRE(n_patches <= n && n < (1LL << 30), CN_ERR_SHAPE, "cn_patch_indices: %d patches of %lld corners",
               n_patches, (long long)n);
    if (n_patches == 0) return CN_OK;
    int hb = 1;
    while ((1LL << (2 * hb)) < n) ++hb;
    patch_indices_kernel<<<(n_patches + 255) / 256, 256, 0, (hipStream_t)stream>>>(h, w, ps, n_patches, hb, key, idx);
    return check_launch("cn_patch_indices");
}

extern "C" int cn_uniform_philox(int64_t n, const uint64_t* seed_offset, float* out, cn_stream_t stream) {
    CN_REQUIRE(n >= 0 && (n == 0 || (seed_offset && out)), CN_ERR_ARG, "cn_uniform_philox: null pointer / n < 0");
    if (n == 0) return CN_OK;
    const int64_t groups = (n + 3) / 4;
    CN_REQUIRE(groups < ((int64_t)1 << 40), CN_ERR_SHAPE, "cn_uniform_philox: n too large");
    uniform_philox_kernel<<<(unsigned)((groups + 255) / 256), 256, 0, (hipStream_t)stream>>>(n, seed_offset, out);
    return check_launch("cn_uniform_philox");
}

extern "C" int cn_coarse_z(int32_t R, int32_t n, const float* near, const float* far, const float* t_rand, float* z,
                           cn_stream_t stream) {
    CN_REQUIRE(near && far && z, CN_ERR_ARG, "cn_coarse_z: null pointer");
    CN_REQUIRE(R >= 0 && n >= 1, CN_ERR_SHAPE, "cn_coarse_z: R=%d n=%d", R, n);
    const int64_t tot = (int64_t)R * n;
    if (tot == 0) return CN_OK;
    coarse_z_kernel<<<(int)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(R, n, near, far, t_rand, z);
    return check_launch("cn_coarse_z");
}

extern "C" int cn_points(int32_t R, int32_t n, const float* rays_o, const float* rays_d, const float* z,
                         const float* t, int32_t mid, const float* near, const float* far, int32_t n_coarse,
                         float* pts_time, cn_stream_t stream) {
    CN_REQUIRE(rays_o && rays_d && z && t && pts_time, CN_ERR_ARG, "cn_points: null pointer");
    CN_REQUIRE(!mid || (near && far && n_coarse > 0), CN_ERR_ARG, "cn_points: mid needs near/far/n_coarse");
    CN_REQUIRE(al16(pts_time), CN_ERR_ALIGN, "cn_points: pts_time alignment");
    const int64_t tot = (int64_t)R * n;
    if (tot == 0) return CN_OK;
    points_kernel<<<(int)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(R, n, rays_o, rays_d, z, t, mid, near, far,
                                                                             n_coarse, pts_time);
    return check_launch("cn_points");
}

extern "C" int cn_points_bwd(int32_t R, int32_t n, const float* z, int32_t mid, const float* near, const float* far,
                             int32_t n_coarse, const float* dP, int64_t ld_p, float* drays_o, float* drays_d,
                             cn_stream_t stream) {
    CN_REQUIRE(z && dP && (drays_o || drays_d), CN_ERR_ARG, "cn_points_bwd: null pointer");
    CN_REQUIRE(!mid || (near && far && n_coarse > 0), CN_ERR_ARG, "cn_points_bwd: mid needs near/far/n_coarse");
    CN_REQUIRE(R >= 0 && n >= 1 && ld_p >= 3, CN_ERR_SHAPE, "cn_points_bwd: R=%d n=%d ld_p=%lld", R, n, (long long)ld_p);
    if (R == 0) return CN_OK;
    points_bwd_kernel<<<cdiv(R, kRaysPerBlock), 64 * kRaysPerBlock, 0, (hipStream_t)stream>>>(
        R, n, z, mid, near, far, n_coarse, dP, ld_p, drays_o, drays_d);
    return check_launch("cn_points_bwd");
}

extern "C" int cn_up_sample_merge(int32_t R, int32_t n, int32_t n_imp, float inv_s, const float* z, const float* sdf,
                                  float* z_out, float* z_new, float* sdf_out, int32_t* new_dst, cn_stream_t stream) {
    CN_REQUIRE(z && sdf && z_out && z_new, CN_ERR_ARG, "cn_up_sample_merge: null pointer");
    CN_REQUIRE(n >= 2 && n_imp >= 1 && n_imp <= 64 && n - 1 <= 64 * kMaxPerLane && n + n_imp <= 256,
               CN_ERR_UNSUPPORTED, "cn_up_sample_merge: n=%d n_imp=%d", n, n_imp);
    if (R == 0) return CN_OK;
    up_sample_merge_kernel<<<cdiv(R, kRaysPerBlock), 64 * kRaysPerBlock, 0, (hipStream_t)stream>>>(
        R, n, n_imp, inv_s, z, sdf, z_out, z_new, sdf_out, new_dst);
    return check_launch("cn_up_sample_merge");
}

extern "C" int cn_composite_fwd(int32_t R, int32_t S, const float* z, const float* sdf, const float* G, int64_t ld_g,
                                const float* rgb, const float* rays_d, const float* inv_s, const float* near,
                                const float* far, int32_t n_coarse, const float* cos_anneal_ratio, float* color, float* depth,
                                float* weights, float* cdf, cn_stream_t stream) {
    CN_REQUIRE(z && sdf && G && rgb && rays_d && inv_s && near && far && cos_anneal_ratio && color && depth && weights,
               CN_ERR_ARG,
               "cn_composite_fwd: null pointer");
    CN_REQUIRE(S >= 1 && S <= 64 * kMaxPerLane && n_coarse > 0 && ld_g >= 3, CN_ERR_UNSUPPORTED,
               "cn_composite_fwd: S=%d", S);
    if (R == 0) return CN_OK;
    composite_fwd_kernel<<<cdiv(R, kRaysPerBlock), 64 * kRaysPerBlock, 0, (hipStream_t)stream>>>(
        R, S, z, sdf, G, ld_g, rgb, rays_d, inv_s, near, far, n_coarse, cos_anneal_ratio, color, depth, weights, cdf);
    return check_launch("cn_composite_fwd");
}

extern "C" int cn_composite_bwd(int32_t R, int32_t S, const float* z, const float* sdf, const float* G, int64_t ld_g,
                                const float* rgb, const float* rays_d, const float* inv_s, const float* near,
                                const float* far, int32_t n_coarse, const float* cos_anneal_ratio, const float* dcolor,
                                const float* ddepth, const float* dweights, const float* dcdf, float* dsdf, float* dG,
                                float* drgb, float* dinv_s_part, float* drays_d, cn_stream_t stream) {
    CN_REQUIRE(z && sdf && G && rgb && rays_d && inv_s && near && far && cos_anneal_ratio && dsdf && dG && drgb &&
                   dinv_s_part,
               CN_ERR_ARG, "cn_composite_bwd: null pointer");
    CN_REQUIRE(S >= 1 && S <= 64 * kMaxPerLane && n_coarse > 0 && ld_g >= 3, CN_ERR_UNSUPPORTED,
               "cn_composite_bwd: S=%d", S);
    if (R == 0) return CN_OK;
    composite_bwd_kernel<<<cdiv(R, kRaysPerBlock), 64 * kRaysPerBlock, 0, (hipStream_t)stream>>>(
        R, S, z, sdf, G, ld_g, rgb, rays_d, inv_s, near, far, n_coarse, cos_anneal_ratio, dcolor, ddepth, dweights,
        dcdf, dsdf, dG, drgb, dinv_s_part, drays_d);
    return check_launch("cn_composite_bwd");
}
