// Shared device helpers for libisr (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <set>
#include <utility>

#include "isr.h"

namespace isr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) float f32x8;

#define ISR_LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

// One 32x32x16 bf16 MFMA: acc += A(32x16) * B(16x32).
// Lane l (r = l & 31, h = l >> 5) supplies A[r][8h..8h+7] and B[8h..8h+7][r];
// accumulator register g of lane l holds D[(g&3) + 8*(g>>2) + 4*h][r].
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 acc) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}

// Storage type of activations and packed weights, a compile-time choice per kernel: H = false →
// bf16 (training, the per-conv backward), H = true → fp16 (the inference path, isr_conv_desc.f16:
// 10 mantissa bits instead of 7 at the same MFMA rate, v_mfma_f32_32x32x16_f16 with the same
// fragment layout).  Fragments travel as 16-byte bf16x8 containers; only the MFMA and the
// float conversions at the epilogue / loads look at the type.
template <bool H>
__device__ __forceinline__ f32x16 mfma32t(bf16x8 a, bf16x8 b, f32x16 acc) {
    if constexpr (H) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc,
                                                      0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
}

// element e of an 8-element storage vector as float
template <bool H>
__device__ __forceinline__ float elt(bf16x8 v, int e) {
    if constexpr (H) return (float)__builtin_bit_cast(f16x8, v)[e];
    else return (float)v[e];
}

// 8 floats → one 16-byte storage vector (round to nearest even)
template <bool H>
__device__ __forceinline__ bf16x8 pack8(const float* x) {
    if constexpr (H) {
        f16x8 t;
#pragma unroll
        for (int e = 0; e < 8; ++e) t[e] = (_Float16)x[e];
        return __builtin_bit_cast(bf16x8, t);
    } else {
        bf16x8 t;
#pragma unroll
        for (int e = 0; e < 8; ++e) t[e] = (__bf16)x[e];
        return t;
    }
}

// the storage bits of one float (16 bits, in the low half)
template <bool H>
__device__ __forceinline__ uint16_t bits16(float x) {
    if constexpr (H) return __builtin_bit_cast(uint16_t, (_Float16)x);
    else return __builtin_bit_cast(uint16_t, (__bf16)x);
}

__device__ __forceinline__ void swap_halves(float& lo, float& hi) {
    // v_permlane32_swap: lanes 32..63 of `lo` trade places with lanes 0..31 of `hi`
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    lo = __uint_as_float(r[0]);
    hi = __uint_as_float(r[1]);
}

__device__ __forceinline__ bf16x8 lds_read16(const char* p) {
    return *reinterpret_cast<const bf16x8*>(p);
}

// ds_read_b128 the compiler does not see as a load: the caller waits for it with its own
// counted `s_waitcnt lgkmcnt(N)` (lds_wait).  For loops where hipcc's waitcnt insertion falls
// back to lgkmcnt(0) before every MFMA.  Compiler-issued LDS ops around these only make the
// counted waits stronger (lgkmcnt(N) retires all but the N youngest, whoever issued them).
__device__ __forceinline__ bf16x8 lds_read16_async(const char* p) {
    bf16x8 r;
    const uint32_t a = (uint32_t)(uintptr_t)ISR_LDS_PTR(p);
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a) : "memory");
    return r;
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8& a, bf16x8& b) {
    static_assert(N >= 0 && N <= 15, "lgkmcnt range");
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
}

// Asynchronous 16-byte-per-lane global → LDS copy (global_load_lds_dwordx4).
// The LDS destination is wave-uniform `lds` + lane*16.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds) {
    __builtin_amdgcn_global_load_lds(gsrc, ISR_LDS_PTR(lds), 16, 0, 0);
}

// The same copy with sc1 (bypasses this CU's L1): reads of activations another workgroup
// of the same launch wrote (cdna_hip_programming.md Guideline 16 hand-offs).
__device__ __forceinline__ void glds16_sc1(const void* gsrc, void* lds) {
    __builtin_amdgcn_global_load_lds(gsrc, ISR_LDS_PTR(lds), 16, 0, 16);
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// Activations are channel-blocked: [N][cs/16][hp][wp][16] bf16 (one 16-channel
// "plane" per block of channels).  Byte address of interior pixel (img, y, x),
// view channel c (c % 8 == 0 for vector accesses).
template <class V>
__device__ __forceinline__ char* view_at(const V& v, int img, int y, int x, int c) {
    const int ch = v.coff + c;
    const size_t plane = (size_t)img * (v.cs >> 4) + (ch >> 4);
    const size_t pix = (plane * v.hp + (y + v.pad)) * (size_t)v.wp + (size_t)(x + v.pad);
    return (char*)v.data + (pix * 16 + (ch & 15)) * 2;
}

// Byte stride between consecutive 16-channel planes of a view.
template <class V>
__device__ __forceinline__ size_t plane_bytes(const V& v) { return (size_t)v.hp * v.wp * 32; }

// Bijective XCD-aware remap of a 1D block id: blocks b and b+8 run on the same
// XCD (round-robin dispatch, MI355X_MICROARCH.md), so give each XCD a
// contiguous range of logical tiles — neighbouring tiles share halo rows in
// that XCD's L2.  Speed only; any placement is correct.
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total >> 3, r = total & 7, x = b & 7, k = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// LDS halo plane image: 2 units of 16 B (8 channels) per pixel, XOR-swizzled
// by bit 3 of the pixel index so that the 32 consecutive pixels of an MFMA A
// fragment (one ds_read_b128 per lane) hit 16 distinct bank slots per lane group.
__device__ __forceinline__ int halo_unit2(int q, int c) { return q * 2 + (c ^ ((q >> 3) & 1)); }

__device__ __forceinline__ void load8_bf16(const char* p, float* v) {
    bf16x8 t = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)t[e];
}

__device__ __forceinline__ void store8_bf16(char* p, const float* v) {
    bf16x8 t;
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = (__bf16)v[e];
    *reinterpret_cast<bf16x8*>(p) = t;
}

template <bool H>
__device__ __forceinline__ void load8_t(const char* p, float* v) {
    const bf16x8 t = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = elt<H>(t, e);
}

template <bool H>
__device__ __forceinline__ void store8_t(char* p, const float* v) {
    *reinterpret_cast<bf16x8*>(p) = pack8<H>(v);
}

// 16-byte load / 8-channel bf16 store at `p` inside view `v`: plain (HX = 0), or the hand-off
// form (HX = 1: sc1 load that bypasses L1; write-through sc1 store, Guideline 16 R1) through a
// buffer descriptor built from the view's base (wave-uniform: no waterfall) with the byte
// offset as the per-lane voffset — hand-off buffers are far below the 2 GiB window.  num_records
// is the view's real extent (n images of cs/16 planes), so a stray offset reads zeros or drops
// the store instead of reaching past the allocation.
template <class V>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const V& v, int n) {
    const size_t bytes = (size_t)n * (v.cs >> 4) * v.hp * v.wp * 32;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(v.data), (short)0,
                                             (int)(bytes < 0x7fffffffull ? bytes : 0x7fffffffull), 0x00020000);
}

template <int HX, class V>
__device__ __forceinline__ bf16x8 load16_hx(const V& v, int n, const char* p) {
    if constexpr (HX) {
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const int off = (int)(p - (const char*)v.data);
        u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(v, n), off, 0, 16);
        return __builtin_bit_cast(bf16x8, r);
    } else {
        return *reinterpret_cast<const bf16x8*>(p);
    }
}

template <int HX, bool H = false, class V>
__device__ __forceinline__ void store8_bf16_hx(const V& v, int n, char* p, const float* x) {
    const bf16x8 t = pack8<H>(x);
    if constexpr (HX) {
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const int off = (int)(p - (const char*)v.data);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, t), rsrc_of(v, n), off, 0, 16);
    } else {
        *reinterpret_cast<bf16x8*>(p) = t;
    }
}

// Fused epilogue on 8 consecutive output channels [co, co+8) of one pixel.
// v = leaky(v + bias); v = v*s1 + r1; v = v*s2 + r2; v *= LeakyReLU'(m) (backward);
// zero outside the valid region.
struct Epi {
    const float* bias;
    float slope, s1, s2;
    isr_view y, y2, r1, r2, m;
    float mslope;
    int h, w;
};

template <bool H = false>
__device__ __forceinline__ void epi_plain8(const Epi& e, float* v, int img, int yy, int xx, int co) {
    if (e.bias) {
        f32x4 b0 = *reinterpret_cast<const f32x4*>(e.bias + co);
        f32x4 b1 = *reinterpret_cast<const f32x4*>(e.bias + co + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) { v[k] += b0[k]; v[4 + k] += b1[k]; }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] >= 0.f ? v[k] : v[k] * e.slope;
    const bool valid = (yy < e.h) && (xx < e.w);
    if (e.r1.data) {
        float r[8];
        load8_t<H>(view_at(e.r1, img, yy, xx, co), r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] * e.s1 + r[k];
    }
    if (e.r2.data) {
        float r[8];
        load8_t<H>(view_at(e.r2, img, yy, xx, co), r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] * e.s2 + r[k];
    }
    if (e.m.data) {
        float m[8];
        load8_t<H>(view_at(e.m, img, yy, xx, co), m);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = m[k] > 0.f ? v[k] : v[k] * e.mslope;
    }
    if (!valid) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = 0.f;
    }
    store8_t<H>(view_at(e.y, img, yy, xx, co), v);
    if (e.y2.data) store8_t<H>(view_at(e.y2, img, yy, xx, co), v);
}

// Raise `kern`'s dynamic-LDS limit to `bytes` once per (kernel, device, host thread).  The
// library is called from the Python thread (forward) and from autograd's device thread
// (backward), and one process may drive several devices; a thread-local record keeps the launch
// path free of locks (hipFuncSetAttribute is idempotent, so each thread setting it once is fine).
inline void lds_limit(const void* kern, int bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    static thread_local std::set<std::pair<const void*, int>> done;
    if (done.insert({kern, dev}).second)
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Compute units of the current device (cached per device, lock-free after the first query).
inline int cu_count() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    static std::atomic<int> cache[64];
    std::atomic<int>& c = cache[dev & 63];
    int v = c.load(std::memory_order_relaxed);
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        c.store(v, std::memory_order_relaxed);
    }
    return v;
}

}  // namespace isr
