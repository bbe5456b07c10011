// 3x3 stride-1 'same' convolution as an implicit GEMM on CDNA4 MFMA
// (v_mfma_f32_32x32x16_bf16), channel-blocked bf16 activations, fp32 accumulation.
//
// Replaces the ATen convolution behind Conv / ConvWithoutBN / RDB / RRDB /
// Scaler of the reference (utils/models.py:75-111, 174-199, 245-271, 298-317,
// 572-589) together with their BN (folded), LeakyReLU, torch.cat, residual
// add/mul and PixelShuffle, which all become the epilogue of one launch.
//
// Block tile: TH = R*WM output rows x 32 output columns x CT = NF*32 output
// channels; wave w owns rows [w*R, w*R+R).  GEMM view per block:
//   M = 32 pixels of one row (one MFMA row-fragment per output row),
//   N = CT output channels (NF fragments of 32),
//   K = 9 taps x Cin, walked in chunks of KC (16 or 32) input channels.
// Activations are [N][C/16][H][W][16]: a K-chunk is KC/16 contiguous planes, so
// each halo row of a chunk is one contiguous 34 x 32-byte run (whole cache
// lines).  Per chunk the (TH+2) x 34 halo planes and the chunk's packed weights
// are copied global → LDS with global_load_lds_dwordx4 into an NST-deep ring;
// each wave walks (k-step, dx) and re-uses every A fragment (one input row) for
// the up-to-3 output rows (dy taps) that read it: R+2 A reads feed 3*R*NF MFMAs.
// The epilogue transposes one output row at a time through LDS so that every
// lane stores 16 contiguous bytes (8 channels) of one pixel.
// Grid: 1D, XCD-aware (xcd_remap) with the cout tile innermost, then x, y, image.
#include "isr_common.h"

namespace isr {

template <int R_, int WM_, int NF_, int KC_, int NST_, int CIN_ = 0>
struct C3 {
    static constexpr int R = R_, WM = WM_, NF = NF_, KC = KC_, NST = NST_;
    static constexpr int CIN = CIN_; // 0 = runtime cin; else compile-time (own symbol)
    static constexpr int TH = R * WM;
    static constexpr int TW = 32;
    static constexpr int HR = TH + 2;  // halo rows
    static constexpr int HC = TW + 2;  // halo cols
    static constexpr int CT = NF * 32; // output channels per block
    static constexpr int KS = KC / 16; // MFMA k-steps (= planes) per chunk
    static constexpr int HQ = HR * HC; // halo pixels per plane
    static constexpr int HIPL = (HQ + 31) / 32; // glds instructions per plane (32 px x 32 B each)
    static constexpr int HALO_INSTR = KS * HIPL;
    static constexpr int W_INSTR = 9 * KS * CT / 32; // [ks][tap][n][hpos] x 16 B
    static constexpr int INSTR = HALO_INSTR + W_INSTR;
    static constexpr int IPW = (INSTR + WM - 1) / WM; // glds per wave per chunk (uniform)
    static constexpr int STAGE = IPW * WM * 1024;
    static constexpr int NT = 64 * WM;
    static constexpr int EPS = CT + 4;                 // floats per pixel in the epilogue image
    static constexpr int EP_BYTES = WM * 32 * EPS * 4; // one output row per wave at a time
    static constexpr int LDS = (NST * STAGE > EP_BYTES) ? NST * STAGE : EP_BYTES;
    static constexpr int BPC = 163840 / LDS; // blocks per CU by LDS
    static constexpr int OCC = BPC * WM / 4 >= 2 ? 2 : 1; // waves per SIMD to budget registers for
    static_assert(LDS <= 163840, "LDS budget");
    static_assert(KC == 16 || KC == 32, "chunk width");
};

// Packed weights (isr_pack_conv3x3): [c16 = cin/16][tap 9][cout][hpos 2][8 bf16],
// element = W[n][c16*16 + h*8 + e][tap], h = hpos ^ ((n >> 3) & 1).
template <class C>
__global__ __launch_bounds__(C::NT, C::OCC) void conv3x3_fwd_kernel(isr_conv_desc d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = C::R, NF = C::NF, WM = C::WM;

    const int nct = d.cout / C::CT;
    const int nbx = d.wa / C::TW, nby = d.ha / C::TH;
    int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ct = t % nct; t /= nct;
    const int bx = t % nbx; t /= nbx;
    const int by = t % nby;
    const int img = t / nby;
    const int x0 = bx * C::TW;
    const int y0 = by * C::TH;
    const int wave = wave_id();
    const int lane = threadIdx.x & 63;
    const int l31 = lane & 31;
    const int hh = lane >> 5;
    const int nchunks = C::CIN ? C::CIN / C::KC : d.cin / C::KC;

    // ---- per-lane glds source offsets (chunk-invariant) -------------------
    const char* xbase = view_at(d.x, img, y0 - 1, x0 - 1, 0);
    const size_t pstride = plane_bytes(d.x);
    const char* wbase = (const char*)d.wpack;
    const int xrow_bytes = d.x.wp * 32;
    const size_t wchunk_bytes = (size_t)C::KS * 9 * d.cout * 32;
    uint32_t off[C::IPW];
#pragma unroll
    for (int k = 0; k < C::IPW; ++k) {
        const int j = wave + WM * k;
        uint32_t o = 0;
        if (j < C::HALO_INSTR) {
            const int kp = j / C::HIPL;
            const int u = (j - kp * C::HIPL) * 64 + lane;
            const int q = u >> 1;
            if (q < C::HQ) {
                const int row = q / C::HC;
                const int col = q - row * C::HC;
                const int c = (u & 1) ^ ((q >> 3) & 1);
                o = (uint32_t)(kp * pstride + row * xrow_bytes + col * 32 + c * 16);
            }
        } else if (j < C::INSTR) {
            const int u = (j - C::HALO_INSTR) * 64 + lane;
            const int seg = u / (C::CT * 2); // (ks, tap)
            const int rem = u - seg * (C::CT * 2);
            o = (uint32_t)((seg * d.cout + ct * C::CT) * 32 + rem * 16);
        }
        off[k] = o;
    }

    auto stage = [&](int chunk, int buf) {
        char* dst = smem + buf * C::STAGE;
        const char* xs = xbase + (size_t)chunk * C::KS * pstride;
        const char* ws = wbase + (size_t)chunk * wchunk_bytes;
#pragma unroll
        for (int k = 0; k < C::IPW; ++k) {
            const int j = wave + WM * k;
            const char* src = (j < C::HALO_INSTR ? xs : ws) + off[k];
            glds16(src, dst + j * 1024);
        }
    };

    f32x16 acc[R][NF];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[r][f][g] = 0.f;

#pragma unroll
    for (int s = 0; s < C::NST - 1; ++s)
        if (s < nchunks) stage(s, s);

    const int qw = wave * R * C::HC + l31; // halo pixel of (row w*R, col l31)
    for (int chunk = 0; chunk < nchunks; ++chunk) {
        // chunk `chunk` landed for this wave: younger chunks in flight = min(NST-2, nchunks-1-chunk)
        if constexpr (C::NST >= 3) {
            if (chunk + C::NST - 2 < nchunks) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((C::NST - 2) * C::IPW) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (chunk + C::NST - 1 < nchunks) stage(chunk + C::NST - 1, (chunk + C::NST - 1) % C::NST);

        const char* hs = smem + (chunk % C::NST) * C::STAGE;
        const char* ws = hs + C::HALO_INSTR * 1024;
#pragma unroll
        for (int ks = 0; ks < C::KS; ++ks) {
            const char* hp = hs + ks * C::HIPL * 1024;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                bf16x8 b[3][NF];
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int f = 0; f < NF; ++f) {
                        const int n = f * 32 + l31;
                        const int u = ((ks * 9 + dy * 3 + dx) * C::CT + n) * 2 + (hh ^ ((n >> 3) & 1));
                        b[dy][f] = lds_read16(ws + u * 16);
                    }
#pragma unroll
                for (int i = 0; i < R + 2; ++i) {
                    const int q = qw + i * C::HC + dx;
                    const bf16x8 a = lds_read16(hp + halo_unit2(q, hh) * 16);
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy) {
                        const int r = i - dy;
                        if (r >= 0 && r < R) {
#pragma unroll
                            for (int f = 0; f < NF; ++f) acc[r][f] = mfma32(a, b[dy][f], acc[r][f]);
                        }
                    }
                }
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier(); // all waves done reading the ring before it becomes the epilogue image

    // ---- epilogue, one output row per pass: acc → LDS [px][CT] fp32 → 8-channel stores
    float* ep = reinterpret_cast<float*>(smem) + wave * (32 * C::EPS);
    Epi e;
    e.bias = d.bias; e.slope = d.slope; e.s1 = d.s1; e.s2 = d.s2;
    e.y = d.y; e.y2 = d.y2; e.r1 = d.r1; e.r2 = d.r2; e.h = d.h; e.w = d.w;
    constexpr int ITEMS = C::CT / 16; // per lane per row
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int px = (g & 3) + 8 * (g >> 2) + 4 * hh;
                ep[px * C::EPS + f * 32 + l31] = acc[r][f][g];
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int yy = y0 + wave * R + r;
        if (d.shuffle == 2) {
            // item → (sub-row si, output col xo in [0,64), 8-channel group cg)
            constexpr int CG = C::CT / 32;
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                const int jj = lane + 64 * it;
                const int cg = jj % CG;
                const int rem = jj / CG;
                const int xo = rem & 63;
                const int si = rem >> 6;
                const int xc = xo >> 1, sj = xo & 1;
                const int xx = x0 + xc;
                float v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int col = 4 * (cg * 8 + k) + 2 * si + sj;
                    v[k] = ep[xc * C::EPS + col] + (e.bias ? e.bias[ct * C::CT + col] : 0.f);
                    v[k] = v[k] >= 0.f ? v[k] : v[k] * e.slope;
                }
                if (!(yy < e.h && xx < e.w)) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = 0.f;
                }
                store8_bf16(view_at(e.y, img, 2 * yy + si, 2 * x0 + xo, ct * (C::CT / 4) + cg * 8), v);
            }
        } else {
            constexpr int CG = C::CT / 8;
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                const int jj = lane + 64 * it;
                const int cg = jj % CG;
                const int px = jj / CG;
                float v[8];
                const float* src = ep + px * C::EPS + cg * 8;
                f32x4 a0 = *reinterpret_cast<const f32x4*>(src);
                f32x4 a1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
                for (int k = 0; k < 4; ++k) { v[k] = a0[k]; v[4 + k] = a1[k]; }
                epi_plain8(e, v, img, yy, x0 + px, ct * C::CT + cg * 8);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
}

template <class C>
static int launch3x3(const isr_conv_desc* d, hipStream_t s) {
    if (d->cout % C::CT || d->cin % C::KC || d->ha % C::TH) return -2;
    if (C::CIN && d->cin != C::CIN) return -2;
    auto kern = conv3x3_fwd_kernel<C>;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
        attr = true;
    }
    const int blocks = (d->wa / C::TW) * (d->ha / C::TH) * d->n * (d->cout / C::CT);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(C::NT), C::LDS, s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Variant table: variant 0 is the production choice per shape; the others are
// kept for on-device A/B tuning (isr_conv3x3_fwd_variant, tools/tune_conv.py).
// cout == 32 (RDB growth convs)
using V_G0 = C3<4, 8, 1, 16, 3>; // 32x32 px tile, 8 waves, 3-deep KC16 ring
using V_G1 = C3<4, 4, 1, 16, 2>; // 16x32, 2 blocks / CU
using V_G2 = C3<2, 4, 1, 32, 2>; // 8x32, KC32, 2 blocks / CU (r1 production)
using V_G3 = C3<2, 8, 1, 16, 3>; // 16x32, 8 waves x 2 rows, 3-deep KC16 ring
// cout % 64 == 0
using V_W0 = C3<4, 8, 2, 16, 2>; // 32x32 px tile, 8 waves, KC16 double buffer
using V_W1 = C3<4, 4, 2, 16, 2>; // 16x32, 2 blocks / CU (r1 production)
using V_W2 = C3<2, 4, 2, 32, 2>; // 8x32, KC32
using V_W3 = C3<4, 4, 2, 32, 2>; // 16x32, KC32, 1 block / CU
using V_F0 = C3<4, 8, 2, 16, 2, 192>; // RDB final conv 192→64: V_W0 with compile-time cin

int conv3x3_fwd_variant(const isr_conv_desc* d, int variant, hipStream_t s) {
    if (d->cout == 32) {
        switch (variant) {
            case 0: return launch3x3<V_G0>(d, s);
            case 1: return launch3x3<V_G1>(d, s);
            case 2: return launch3x3<V_G2>(d, s);
            case 3: return launch3x3<V_G3>(d, s);
        }
        return -2;
    }
    switch (variant) {
        case 0: return d->cin == 192 ? launch3x3<V_F0>(d, s) : launch3x3<V_W0>(d, s);
        case 1: return launch3x3<V_W1>(d, s);
        case 2: return launch3x3<V_W2>(d, s);
        case 3: return launch3x3<V_W3>(d, s);
    }
    return -2;
}

int conv3x3_fwd_dispatch(const isr_conv_desc* d, hipStream_t s) { return conv3x3_fwd_variant(d, 0, s); }

// ---- weight packing: fp32 OIHW → bf16 [c16][tap][cout][hpos][8] -----------
__global__ void pack3x3_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int cout, int cin) {
    const size_t total = (size_t)cout * cin * 9;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
        size_t rem = idx;
        const int e = rem % 8; rem /= 8;
        const int hpos = rem % 2; rem /= 2;
        const int n = rem % cout; rem /= cout;
        const int tap = rem % 9; rem /= 9;
        const int c16 = (int)rem;
        const int h = hpos ^ ((n >> 3) & 1);
        const int ci = c16 * 16 + h * 8 + e;
        out[idx] = (__bf16)w[((size_t)n * cin + ci) * 9 + tap];
    }
}

size_t conv3x3_packed_bytes(int cout, int cin) { return (size_t)cout * cin * 9 * 2; }

int conv3x3_pack(const float* w, void* out, int cout, int cin, hipStream_t s) {
    const size_t total = conv3x3_packed_bytes(cout, cin) / 2;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(pack3x3_kernel, dim3(blocks), dim3(256), 0, s, w, (__bf16*)out, cout, cin);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr
