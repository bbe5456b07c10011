// Multi-tensor optimiser kernels: one launch per step over every parameter of a
// model, replacing the reference's per-tensor loops:
//   Adam step            torch.optim.Adam (train.py:264-267, stepped at :58, :102, :118)
//   clip_grad_norm_(10)  train.py:57, :101, :116 (sum of squares + coefficient + scale)
//   ModelEMA.update      utils/models.py:31-40 (v = v*d + (1-d)*m over the float state_dict)
// Work is a list of chunks (tensor index, start, length) built by the host; a
// block owns one chunk and streams it with 16-byte accesses (HBM-bound).
#include "isr_common.h"

namespace isr {

constexpr int MT_THREADS = 256;

__device__ __forceinline__ bool mt_vec_ok(const isr_mt_tensor& t, int64_t start) {
    // float4 path: every used pointer 16-B aligned at the chunk start
    const uintptr_t a = (uintptr_t)(t.p + start) | (uintptr_t)(t.g ? t.g + start : nullptr) |
                        (uintptr_t)(t.m ? t.m + start : nullptr) | (uintptr_t)(t.v ? t.v + start : nullptr);
    return (a & 15) == 0;
}

struct AdamOp {
    isr_adam_args a;
    const float* scale;
    __device__ __forceinline__ void operator()(float& p, float g, float& m, float& v, float s) const {
        g *= s;
        if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, p, g);
        // exp_avg.lerp_(grad, 1 - beta1) (torch's lerp: weight < 0.5 form)
        m = fmaf(1.f - a.beta1, g - m, m);
        v = fmaf(1.f - a.beta2, g * g, v * a.beta2);
        const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
        p = fmaf(a.step, m / denom, p);  // step = -lr / bias_correction1
    }
};

// guard (nullable): two words written by an earlier launch of the stream (the trunk kernel's
// sticky give-up count and the count the host has accepted, isr_chain_desc state[2] / [3]);
// a block skips its chunk when they differ, so a failed forward never reaches the parameters.
__device__ __forceinline__ bool mt_guarded_out(const uint32_t* guard) {
    return guard != nullptr && guard[0] != guard[1];
}

__global__ __launch_bounds__(MT_THREADS) void mt_adam_kernel(const isr_mt_tensor* __restrict__ ts,
                                                             const isr_mt_chunk* __restrict__ cs, AdamOp op,
                                                             const uint32_t* __restrict__ guard) {
    if (mt_guarded_out(guard)) return;
    const isr_mt_chunk c = cs[blockIdx.x];
    const isr_mt_tensor t = ts[c.t];
    const float s = op.scale ? *op.scale : 1.f;
    if (mt_vec_ok(t, c.start) && (c.len & 3) == 0) {
        float4* p = reinterpret_cast<float4*>(t.p + c.start);
        const float4* g = reinterpret_cast<const float4*>(t.g + c.start);
        float4* m = reinterpret_cast<float4*>(t.m + c.start);
        float4* v = reinterpret_cast<float4*>(t.v + c.start);
        for (int i = threadIdx.x; i < c.len / 4; i += MT_THREADS) {
            float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
            op(pp.x, gg.x, mm.x, vv.x, s);
            op(pp.y, gg.y, mm.y, vv.y, s);
            op(pp.z, gg.z, mm.z, vv.z, s);
            op(pp.w, gg.w, mm.w, vv.w, s);
            p[i] = pp; m[i] = mm; v[i] = vv;
        }
    } else {
        for (int i = threadIdx.x; i < c.len; i += MT_THREADS) {
            const int64_t k = c.start + i;
            float pp = t.p[k], mm = t.m[k], vv = t.v[k];
            op(pp, t.g[k], mm, vv, s);
            t.p[k] = pp; t.m[k] = mm; t.v[k] = vv;
        }
    }
}

// per-chunk sum of squares of g (fp32 partial per chunk)
__global__ __launch_bounds__(MT_THREADS) void mt_sumsq_kernel(const isr_mt_tensor* __restrict__ ts,
                                                              const isr_mt_chunk* __restrict__ cs,
                                                              float* __restrict__ partial) {
    const isr_mt_chunk c = cs[blockIdx.x];
    const float* g = ts[c.t].g + c.start;
    float acc = 0.f;
    if (((uintptr_t)g & 15) == 0 && (c.len & 3) == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(g);
        for (int i = threadIdx.x; i < c.len / 4; i += MT_THREADS) {
            const float4 x = g4[i];
            acc = fmaf(x.x, x.x, acc);
            acc = fmaf(x.y, x.y, acc);
            acc = fmaf(x.z, x.z, acc);
            acc = fmaf(x.w, x.w, acc);
        }
    } else {
        for (int i = threadIdx.x; i < c.len; i += MT_THREADS) acc = fmaf(g[i], g[i], acc);
    }
    __shared__ float red[MT_THREADS / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < MT_THREADS / 64; ++w) s += red[w];
        partial[blockIdx.x] = s;
    }
}

// total_norm = sqrt(sum partial) (double accumulation); coef = min(1, max_norm / (total_norm + 1e-6))
__global__ __launch_bounds__(MT_THREADS) void clip_coef_kernel(const float* __restrict__ partial, int n,
                                                               float max_norm, float* __restrict__ out) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += MT_THREADS) acc += partial[i];
    __shared__ double red[MT_THREADS / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < MT_THREADS / 64; ++w) s += red[w];
        const float norm = (float)sqrt(s);
        const float coef = max_norm / (norm + 1e-6f);
        out[0] = norm;
        out[1] = coef < 1.f ? coef : 1.f;
    }
}

// g *= *coef  (mode 0)   |   p = p*d + (1-d)*g  (mode 1: EMA, p = ema tensor, g = model tensor)
__global__ __launch_bounds__(MT_THREADS) void mt_axpby_kernel(const isr_mt_tensor* __restrict__ ts,
                                                              const isr_mt_chunk* __restrict__ cs, int mode,
                                                              const float* __restrict__ coef, float d,
                                                              const uint32_t* __restrict__ guard) {
    if (mt_guarded_out(guard)) return;
    const isr_mt_chunk c = cs[blockIdx.x];
    const isr_mt_tensor t = ts[c.t];
    if (mode == 0) {
        const float k = *coef;
        float* g = t.g + c.start;
        if (((uintptr_t)g & 15) == 0 && (c.len & 3) == 0) {
            float4* g4 = reinterpret_cast<float4*>(g);
            for (int i = threadIdx.x; i < c.len / 4; i += MT_THREADS) {
                float4 x = g4[i];
                x.x *= k; x.y *= k; x.z *= k; x.w *= k;
                g4[i] = x;
            }
        } else {
            for (int i = threadIdx.x; i < c.len; i += MT_THREADS) g[i] *= k;
        }
    } else {
        const float e = 1.f - d;
        float* p = t.p + c.start;
        const float* g = t.g + c.start;
        if ((((uintptr_t)p | (uintptr_t)g) & 15) == 0 && (c.len & 3) == 0) {
            float4* p4 = reinterpret_cast<float4*>(p);
            const float4* g4 = reinterpret_cast<const float4*>(g);
            for (int i = threadIdx.x; i < c.len / 4; i += MT_THREADS) {
                float4 x = p4[i];
                const float4 y = g4[i];
                x.x = x.x * d + y.x * e; x.y = x.y * d + y.y * e;
                x.z = x.z * d + y.z * e; x.w = x.w * d + y.w * e;
                p4[i] = x;
            }
        } else {
            for (int i = threadIdx.x; i < c.len; i += MT_THREADS) p[i] = p[i] * d + g[i] * e;
        }
    }
}

int mt_adam_dispatch(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int n, const isr_adam_args* a,
                     const float* scale, const uint32_t* guard, hipStream_t s) {
    hipLaunchKernelGGL(mt_adam_kernel, dim3(n), dim3(MT_THREADS), 0, s, ts, cs, AdamOp{*a, scale}, guard);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int mt_sumsq_dispatch(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int n, float* partial, hipStream_t s) {
    hipLaunchKernelGGL(mt_sumsq_kernel, dim3(n), dim3(MT_THREADS), 0, s, ts, cs, partial);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int clip_coef_dispatch(const float* partial, int n, float max_norm, float* out, hipStream_t s) {
    hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(MT_THREADS), 0, s, partial, n, max_norm, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int mt_axpby_dispatch(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int n, int mode, const float* coef, float d,
                      const uint32_t* guard, hipStream_t s) {
    hipLaunchKernelGGL(mt_axpby_kernel, dim3(n), dim3(MT_THREADS), 0, s, ts, cs, mode, coef, d, guard);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr
