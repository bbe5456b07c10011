// Elementwise glue on channel-blocked bf16 views (see isr_ew_desc in isr.h).
// One thread per (pixel, 8 channels): 16-byte loads/stores, whole computed
// region (ha x wa), zeros written outside the valid h x w region.
#include "isr_common.h"

// Index type of the grid-stride elementwise kernels: 32-bit (cheap div/mod for the
// pixel decomposition) whenever the element-group count leaves headroom for the stride.
#define ISR_IDX_LAUNCH(K, total, grid, s, arg)                                          \
    do {                                                                                \
        if ((size_t)(total) < (1ull << 31)) hipLaunchKernelGGL(K<uint32_t>, grid, dim3(256), 0, s, arg); \
        else hipLaunchKernelGGL(K<size_t>, grid, dim3(256), 0, s, arg);                \
    } while (0)

namespace isr {

template <typename I>
__global__ __launch_bounds__(256) void ew_combine_kernel(isr_ew_desc d) {
    const int cg = d.c / 8;
    const I total = (I)((size_t)d.n * d.ha * d.wa * cg);
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        // channel group innermost within a 16-channel plane pair, then x, y, plane, image:
        // consecutive threads touch consecutive 16-byte units of one plane row.
        I r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y < d.h && x < d.w) {
            float t[8];
            load8_bf16(view_at(d.a, img, y, x, c), t);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = t[k] * d.sa;
            if (d.b.data) {
                load8_bf16(view_at(d.b, img, y, x, c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] += t[k] * d.sb;
            }
            if (d.m.data) {
                load8_bf16(view_at(d.m, img, y, x, c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = t[k] > 0.f ? v[k] : v[k] * d.mslope;
            }
        }
        store8_bf16(view_at(d.y, img, y, x, c), v);
    }
}

int ew_combine_dispatch(const isr_ew_desc* d, hipStream_t s) {
    const size_t total = (size_t)d->n * d->ha * d->wa * (d->c / 8);
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    ISR_IDX_LAUNCH(ew_combine_kernel, total, dim3(blocks), s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// PixelShuffle(2) + LeakyReLU between channel-blocked views (isr_pixel_shuffle2):
// y[c] at (y, x) = act(sa * a[4c + 2(y&1) + (x&1)] at (y/2, x/2)).  One thread per
// (output pixel, 8 output channels): the 8 source channels 4c+s .. 4c+28+s are
// gathered from the 32 channels (two 16-channel planes) at the source pixel; the
// four sub-pixel threads of a source pixel re-read the same 64 bytes from L2.
template <typename I>
__global__ __launch_bounds__(256) void pixel_shuffle2_kernel(isr_ew_desc d) {
    const int cg = d.c / 8;
    const I total = (I)((size_t)d.n * d.ha * d.wa * cg);
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y < d.h && x < d.w) {
            const int s = 2 * (y & 1) + (x & 1);
            float t[32];
#pragma unroll
            for (int q = 0; q < 4; ++q) load8_bf16(view_at(d.a, img, y >> 1, x >> 1, 4 * c + 8 * q), t + 8 * q);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float u = t[4 * k + s] * d.sa;
                v[k] = u > 0.f ? u : u * d.mslope;
            }
        }
        store8_bf16(view_at(d.y, img, y, x, c), v);
    }
}

// Its transpose (isr_pixel_unshuffle2): y[4c + s] at (y, x) = sa * a[c] at (2y + s/2, 2x + s%2),
// times LeakyReLU'(m) there when m is given.  One thread per (output pixel, 8 source
// channels): four 16-byte source loads (one per sub-pixel), four 16-byte stores of the
// 32 output channels 4c0 .. 4c0 + 31.
template <typename I>
__global__ __launch_bounds__(256) void pixel_unshuffle2_kernel(isr_ew_desc d) {
    const int cg = d.c / 32;
    const I total = (I)((size_t)d.n * d.ha * d.wa * cg);
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int g = r % cg;
        const int img = (int)(r / cg);
        const int c0 = g * 8;  // first source channel
        float t[4][8];
        if (y < d.h && x < d.w) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int yy = 2 * y + (s >> 1), xx = 2 * x + (s & 1);
                load8_bf16(view_at(d.a, img, yy, xx, c0), t[s]);
                float mm[8];
                if (d.m.data) load8_bf16(view_at(d.m, img, yy, xx, c0), mm);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    t[s][k] *= d.sa;
                    if (d.m.data && !(mm[k] > 0.f)) t[s][k] *= d.mslope;
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int k = 0; k < 8; ++k) t[s][k] = 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // output channels 4c0 + 8q .. +7 = (c0 + 2q + j/4, s = j%4)
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = t[j & 3][2 * q + (j >> 2)];
            store8_bf16(view_at(d.y, img, y, x, 4 * c0 + 8 * q), v);
        }
    }
}

int pixel_unshuffle2_dispatch(const isr_ew_desc* d, hipStream_t s) {
    const size_t total = (size_t)d->n * d->ha * d->wa * (d->c / 32);
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    ISR_IDX_LAUNCH(pixel_unshuffle2_kernel, total, dim3(blocks), s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int pixel_shuffle2_dispatch(const isr_ew_desc* d, hipStream_t s) {
    const size_t total = (size_t)d->n * d->ha * d->wa * (d->c / 8);
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    ISR_IDX_LAUNCH(pixel_shuffle2_kernel, total, dim3(blocks), s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr

namespace isr {

// NCHW fp32 → channel-blocked bf16 (channels [0, round16(c)), zero padded), with
// optional per-channel affine and LeakyReLU' mask; zeros outside the valid region.
template <typename I>
__global__ __launch_bounds__(256) void nchw_to_blocked_kernel(isr_convert_desc d) {
    const int cp = (d.c + 15) / 16;
    const I total = (I)((size_t)d.n * cp * d.ha * d.wa);
    const size_t plane = (size_t)d.h * d.w;
    const float* src = (const float*)d.nchw;
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int pl = r % cp;
        const int img = (int)(r / cp);
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = 0.f;
        const bool valid = y < d.h && x < d.w;
        if (valid) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int c = pl * 16 + k;
                if (c < d.c) {
                    float t = src[((size_t)img * d.c + c) * plane + (size_t)y * d.w + x];
                    if (d.scale) t *= d.scale[c];
                    if (d.shift) t += d.shift[c];
                    v[k] = t;
                }
            }
            if (d.m.data) {
                float m[8];
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    load8_bf16(view_at(d.m, img, y, x, pl * 16 + hf * 8), m);
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[hf * 8 + k] = m[k] > 0.f ? v[hf * 8 + k] : v[hf * 8 + k] * d.mslope;
                }
            }
        }
        char* p = view_at(d.v, img, y, x, pl * 16);
        store8_bf16(p, v);
        store8_bf16(p + 16, v + 8);
    }
}

// channel-blocked bf16 → NCHW fp32 (channels [0, c), valid region only)
template <typename I>
__global__ __launch_bounds__(256) void blocked_to_nchw_kernel(isr_convert_desc d) {
    const I total = (I)((size_t)d.n * d.c * d.h * d.w);
    const size_t plane = (size_t)d.h * d.w;
    float* dst = (float*)d.nchw;
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        const int x = (int)(i % d.w);
        const int y = (int)((i / d.w) % d.h);
        const size_t ic = i / plane;
        const int c = (int)(ic % d.c), img = (int)(ic / d.c);
        const __bf16 v = *reinterpret_cast<const __bf16*>(view_at(d.v, img, y, x, c));
        float t = (float)v;
        if (d.scale) t *= d.scale[c];
        if (d.shift) t += d.shift[c];
        dst[i] = t;
    }
}

// 2x2 / stride-2 max pool on blocked views (utils/models.py:454-510 via torchvision
// vgg19.features MaxPool2d(2, 2)); output grid (h/2, w/2), computed region (ha_o, wa_o).
template <typename I>
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(isr_pool_desc d) {
    const int cg = d.c / 8;
    const int ho = d.h / 2, wo = d.w / 2;
    const I total = (I)((size_t)d.n * d.hao * d.wao * cg);
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wao; r /= d.wao;
        const int y = r % d.hao; r /= d.hao;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y < ho && x < wo) {
            float t[8];
            load8_bf16(view_at(d.x, img, 2 * y, 2 * x, c), v);
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                load8_bf16(view_at(d.x, img, 2 * y + (q >> 1), 2 * x + (q & 1), c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = t[k] > v[k] ? t[k] : v[k];
            }
        }
        store8_bf16(view_at(d.y, img, y, x, c), v);
    }
}

// backward: g_in at the first maximum of each window (PyTorch's scan order, row-major)
// = g_out, times (x > 0 ? 1 : mslope) — the ReLU' of the layer that produced x.
template <typename I>
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(isr_pool_desc d) {
    const int cg = d.c / 8;
    const int ho = d.h / 2, wo = d.w / 2;
    const I total = (I)((size_t)d.n * d.hao * d.wao * cg);
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wao; r /= d.wao;
        const int y = r % d.hao; r /= d.hao;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float win[4][8], go[8], best[8];
        int arg[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) load8_bf16(view_at(d.x, img, 2 * y + (q >> 1), 2 * x + (q & 1), c), win[q]);
        const bool valid = y < ho && x < wo;
        if (valid) load8_bf16(view_at(d.y, img, y, x, c), go);
#pragma unroll
        for (int k = 0; k < 8; ++k) { best[k] = win[0][k]; arg[k] = 0; }
#pragma unroll
        for (int q = 1; q < 4; ++q)
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (win[q][k] > best[k]) { best[k] = win[q][k]; arg[k] = q; }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float o[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float gk = (valid && arg[k] == q) ? go[k] : 0.f;
                o[k] = win[q][k] > 0.f ? gk : gk * d.mslope;
            }
            store8_bf16(view_at(d.g, img, 2 * y + (q >> 1), 2 * x + (q & 1), c), o);
        }
    }
}

static int blocks_for(size_t total) { return (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192); }

int nchw_to_blocked_dispatch(const isr_convert_desc* d, hipStream_t s) {
    const size_t total = (size_t)d->n * ((d->c + 15) / 16) * d->ha * d->wa;
    ISR_IDX_LAUNCH(nchw_to_blocked_kernel, total, dim3(blocks_for(total)), s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int blocked_to_nchw_dispatch(const isr_convert_desc* d, hipStream_t s) {
    const size_t total = (size_t)d->n * d->c * d->h * d->w;
    ISR_IDX_LAUNCH(blocked_to_nchw_kernel, total, dim3(blocks_for(total)), s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int maxpool2_dispatch(const isr_pool_desc* d, int backward, hipStream_t s) {
    const size_t total = (size_t)d->n * d->hao * d->wao * (d->c / 8);
    if (backward) ISR_IDX_LAUNCH(maxpool2_bwd_kernel, total, dim3(blocks_for(total)), s, *d);
    else ISR_IDX_LAUNCH(maxpool2_fwd_kernel, total, dim3(blocks_for(total)), s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr

// ------------------------------------------------------------------ BatchNorm
// Train-mode BatchNorm2d on channel-blocked views (the `bn` of Conv,
// utils/models.py:75-111, in ResNet's train mode).  Statistics over (N, H, W)
// per channel accumulate in double (caller-zeroed acc[2][c]); the per-thread
// and per-block partials are fp32 over at most a few thousand values.
namespace isr {

constexpr int BN_ROWS = 8;  // rows of one plane per block

// (sum, sumsq) of z  [mode 0]  or  (sum g, sum g*xhat) [mode 1] per channel
template <int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(isr_bn_desc d) {
    __shared__ float red[4][2][16];
    const int planes = d.c / 16;
    const int nrb = (d.h + BN_ROWS - 1) / BN_ROWS;
    int b = blockIdx.x;
    const int rb = b % nrb; b /= nrb;
    const int pl = b % planes;
    const int img = b / planes;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int half = threadIdx.x & 1;
    const int c0 = pl * 16 + half * 8;
    float s1[8], s2[8], mean[8], istd[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s1[k] = 0.f;
        s2[k] = 0.f;
        if (MODE == 1) { mean[k] = d.save[c0 + k]; istd[k] = d.save[d.c + c0 + k]; }
    }
    const int y0 = rb * BN_ROWS, y1 = min(d.h, y0 + BN_ROWS);
    for (int y = y0; y < y1; ++y) {
        for (int x = threadIdx.x >> 1; x < d.w; x += 128) {
            float z[8];
            load8_bf16(view_at(d.z, img, y, x, c0), z);
            if (MODE == 0) {
#pragma unroll
                for (int k = 0; k < 8; ++k) { s1[k] += z[k]; s2[k] += z[k] * z[k]; }
            } else {
                float g[8];
                load8_bf16(view_at(d.y, img, y, x, c0), g);
#pragma unroll
                for (int k = 0; k < 8; ++k) { s1[k] += g[k]; s2[k] += g[k] * (z[k] - mean[k]) * istd[k]; }
            }
        }
    }
    // reduce over the 32 lanes of equal parity
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int o = 2; o < 64; o <<= 1) {
            s1[k] += __shfl_xor(s1[k], o);
            s2[k] += __shfl_xor(s2[k], o);
        }
    }
    if (lane < 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { red[wave][0][half * 8 + k] = s1[k]; red[wave][1][half * 8 + k] = s2[k]; }
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        const int q = threadIdx.x >> 4, ch = threadIdx.x & 15;
        const float v = red[0][q][ch] + red[1][q][ch] + red[2][q][ch] + red[3][q][ch];
        atomicAdd(d.acc + q * d.c + pl * 16 + ch, (double)v);
    }
}

// forward finalize: save = (mean, invstd); running stats (unbiased var), as nn.BatchNorm2d.train()
__global__ void bn_finalize_kernel(isr_bn_desc d) {
    const double cnt = (double)d.n * d.h * d.w;
    for (int c = threadIdx.x; c < d.c; c += blockDim.x) {
        const double mean = d.acc[c] / cnt;
        double var = d.acc[d.c + c] / cnt - mean * mean;
        var = var > 0.0 ? var : 0.0;
        d.save[c] = (float)mean;
        d.save[d.c + c] = (float)(1.0 / sqrt(var + (double)d.eps));
        if (d.running_mean) {
            d.running_mean[c] = (1.f - d.momentum) * d.running_mean[c] + d.momentum * (float)mean;
            d.running_var[c] = (1.f - d.momentum) * d.running_var[c] + d.momentum * (float)(var * cnt / (cnt > 1 ? cnt - 1 : 1));
        }
    }
}

// y = ((act(a*z + b)) * s1 + r1) * s2 + r2;  a = gamma*invstd, b = beta - mean*a
template <typename I>
#define BN_MAX_C 1024  // channels per BatchNorm layer (validated on the host)

__global__ __launch_bounds__(256) void bn_apply_kernel(isr_bn_desc d) {
    // per-channel affine (a, b) once per block in LDS: the element loop is one FMA per value
    __shared__ float ca[BN_MAX_C], cb[BN_MAX_C];
    for (int c = threadIdx.x; c < d.c; c += blockDim.x) {
        const float a = d.gamma[c] * d.save[d.c + c];
        ca[c] = a;
        cb[c] = d.beta[c] - d.save[c] * a;
    }
    __syncthreads();
    const int cg = d.c / 8;
    const I total = (I)((size_t)d.n * d.ha * d.wa * cg);
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y < d.h && x < d.w) {
            load8_bf16(view_at(d.z, img, y, x, c), v);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float t = v[k] * ca[c + k] + cb[c + k];
                t = t >= 0.f ? t : t * d.slope;
                v[k] = t * d.s1;
            }
            if (d.r1.data) {
                float t[8];
                load8_bf16(view_at(d.r1, img, y, x, c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] += t[k];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] *= d.s2;
            if (d.r2.data) {
                float t[8];
                load8_bf16(view_at(d.r2, img, y, x, c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] += t[k];
            }
        }
        store8_bf16(view_at(d.y, img, y, x, c), v);
    }
}

// dz = gscale * a * (g - sum(g)/N - xhat * sum(g*xhat)/N), in place over y; dgamma/dbeta
template <typename I>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(isr_bn_desc d) {
    // dz = gs*gamma*istd * (g - mean(g) - xhat * mean(g*xhat)) = A*(g - mg) - K*(z - mean) per
    // channel, with A, mg, K = A*istd*mean(g*xhat) and the mean computed once per block in LDS (the
    // element loop had two fp64 divides per value).  The subtraction z - mean is kept explicit: a
    // folded B*z + C form cancels in fp32 when |mean| >> std.
    __shared__ float ca[BN_MAX_C], cb[BN_MAX_C], cc[BN_MAX_C], cm[BN_MAX_C];
    const int cg = d.c / 8;
    const I total = (I)((size_t)d.n * d.ha * d.wa * cg);
    const double cnt = (double)d.n * d.h * d.w;
    for (int c = threadIdx.x; c < d.c; c += blockDim.x) {
        const float mean = d.save[c], istd = d.save[d.c + c];
        const float mg = (float)(d.acc[c] / cnt), mgx = (float)(d.acc[d.c + c] / cnt);
        const float A = d.gscale * d.gamma[c] * istd;
        ca[c] = A;
        cb[c] = A * istd * mgx;
        cc[c] = mg;
        cm[c] = mean;
    }
    __syncthreads();
    if (blockIdx.x == 0) {
        for (int c = threadIdx.x; c < d.c; c += blockDim.x) {
            if (d.dgamma) d.dgamma[c] = (float)(d.acc[d.c + c]) * d.gscale;
            if (d.dbeta) d.dbeta[c] = (float)(d.acc[c]) * d.gscale;
        }
    }
    for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
        I r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y < d.h && x < d.w) {
            float z[8], g[8];
            load8_bf16(view_at(d.z, img, y, x, c), z);
            load8_bf16(view_at(d.y, img, y, x, c), g);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = ca[c + k] * (g[k] - cc[c + k]) - cb[c + k] * (z[k] - cm[c + k]);
        }
        store8_bf16(view_at(d.dz.data ? d.dz : d.y, img, y, x, c), v);
    }
}

int bn_dispatch(const isr_bn_desc* d, int op, hipStream_t s) {
    const size_t total = (size_t)d->n * d->ha * d->wa * (d->c / 8);
    const int ew_blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    const int red_blocks = d->n * (d->c / 16) * ((d->h + BN_ROWS - 1) / BN_ROWS);
    switch (op) {
        case 0: hipLaunchKernelGGL(bn_reduce_kernel<0>, dim3(red_blocks), dim3(256), 0, s, *d); break;
        case 1: hipLaunchKernelGGL(bn_finalize_kernel, dim3(1), dim3(256), 0, s, *d); break;
        case 2: ISR_IDX_LAUNCH(bn_apply_kernel, total, dim3(ew_blocks), s, *d); break;
        case 3: hipLaunchKernelGGL(bn_reduce_kernel<1>, dim3(red_blocks), dim3(256), 0, s, *d); break;
        case 4: ISR_IDX_LAUNCH(bn_bwd_apply_kernel, total, dim3(ew_blocks), s, *d); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr

namespace isr {

// SR_dataset's per-sample transform (utils/datasets.py:344-355), batched on the device in ONE
// pass over the uint8 crops: one thread per (image, LR pixel) reads its scale x scale HR block of
// every channel, writes those HR pixels (PIL_to_tanh 2x/255 - 1, or Normalize in SRGAN mode) and
// the LR pixel: OpenCV's uint8 INTER_LINEAR resize at an integer factor (odd: the block's centre
// pixel; even: its centre 2x2 mean rounded half up — cv2's 11-bit fixed point at weights 0 / 0.5 /
// 1, oracle.ref_cpu.cv2_resize_linear_u8; x2 is cv2's INTER_AREA, the same 2x2 mean), then
// Normalize.  Same float formulas as data.GPUTransform's CPU form.
template <int S>
__global__ __launch_bounds__(256) void sr_transform_kernel(isr_sr_transform_desc d) {
    const int t = d.t, lt = t / S;
    const uint32_t total = (uint32_t)d.n * lt * lt;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const int lx = (int)(i % lt), tmp = (int)(i / lt), ly = tmp % lt, img = tmp / lt;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const size_t plane = (size_t)img * 3 + c;
            const uint8_t* src = d.crops + (plane * t + (size_t)ly * S) * t + (size_t)lx * S;
            float* hr = d.hr + (plane * t + (size_t)ly * S) * t + (size_t)lx * S;
            const float mean = d.mean[c], stdv = d.std[c];
            uint32_t u[S][S];
#pragma unroll
            for (int r = 0; r < S; ++r) {
#pragma unroll
                for (int k = 0; k < S; ++k) u[r][k] = src[(size_t)r * t + k];
#pragma unroll
                for (int k = 0; k < S; ++k) {
                    const float x = (float)u[r][k] / 255.f;
                    hr[(size_t)r * t + k] = d.hr_norm ? (x - mean) / stdv : x * 2.f - 1.f;
                }
            }
            uint32_t q;
            if constexpr (S % 2 == 1) {
                q = u[(S - 1) / 2][(S - 1) / 2];
            } else {
                constexpr int c0 = S / 2 - 1;
                q = (u[c0][c0] + u[c0][c0 + 1] + u[c0 + 1][c0] + u[c0 + 1][c0 + 1] + 2u) >> 2;
            }
            d.lr[(plane * lt + ly) * lt + lx] = ((float)q / 255.f - mean) / stdv;
        }
    }
}

int sr_transform_dispatch(const isr_sr_transform_desc* d, hipStream_t s) {
    const size_t lt = (size_t)(d->t / d->scale), total = (size_t)d->n * lt * lt;
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    switch (d->scale) {
        case 2: hipLaunchKernelGGL(sr_transform_kernel<2>, dim3(blocks), dim3(256), 0, s, *d); break;
        case 3: hipLaunchKernelGGL(sr_transform_kernel<3>, dim3(blocks), dim3(256), 0, s, *d); break;
        case 4: hipLaunchKernelGGL(sr_transform_kernel<4>, dim3(blocks), dim3(256), 0, s, *d); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr
