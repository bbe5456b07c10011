// Weight (and bias) gradient of a 3x3 'same' conv on CDNA4 MFMA — the
// bwd-weight half of autograd through Conv / ConvWithoutBN / RDB / Scaler
// (utils/models.py:75-111, 174-199, 245-271, 572-589; backward of train.py:57, :102).
//
//   dW[co][ci][dy][dx] = scale * sum_{n,y,x} G[n][co][y][x] * X[n][ci][y+dy-1][x+dx-1]
//   db[co]             = scale * sum_{n,y,x} G[n][co][y][x]
//
// GEMM view: M = cout (from G), N = cin (from X, shifted per tap), K = pixels.
// Both operands are channel-blocked [N][C/16][H][W][16] bf16, i.e. pixel-major
// with 16 channels per 32-byte unit, while the MFMA wants 8 consecutive K
// (pixels) per lane for one M/N index (channel): tiles are staged to LDS
// unchanged (global_load_lds, lane-linear) and read with ds_read_b64_tr_b16,
// the gfx950 transposing LDS read (cdna_hip_programming.md T10), which turns a
// [pixel][channel] image into per-channel pixel runs for free.
//
// Block = 3 waves; wave w owns kernel row dy = w and all three dx taps, for a
// CO_T x CI_T (co, ci) tile: 3 * NCO * NCI accumulators of 32x32.  The A
// fragment (G, 32 co x 16 px) is reused by the 3 taps of the wave; the B
// fragment (X shifted by (dy, dx)) is read per tap.  Pixel tiles are TY rows x
// 32 columns; each block walks a contiguous range of them (split-K over
// n*h*w), double-buffered through LDS.  Per-block partial sums go to a
// workspace [split][tap][co][ci | + co bias]; a second kernel
// reduces over splits, applies `scale`, and writes dW in the reference OIHW
// layout (and un-permutes the PixelShuffle channel order for g_sub2).
#include "isr_common.h"
#include <cstdlib>
#include <utility>

namespace isr {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group passes the address of
// pixel-row q, channels 4p..4p+3; lane i of the group receives channel i of
// the 4 pixels.
__device__ __forceinline__ bf16x4 lds_tr4(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p));
}

__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) {
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// The same transposing read as inline asm at base + OFF, which hipcc does not see as an LDS load:
// its waitcnt pass puts a vmcnt(0) in front of the first compiler-visible LDS read after a
// global_load_lds (it cannot tell the stage being read from the one being filled), which made
// every stage wait for the NEXT stage's DMA before computing.  The row sweep waits for these with
// counted lgkmcnt waits of its own (lgk_wait) and ties the fragments to them (tie).
template <int OFF>
__device__ __forceinline__ bf16x4 tr4_at(uint32_t base) {
    bf16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(OFF) : "memory");
    return r;
}
template <int N>
__device__ __forceinline__ void lgk_wait() {
    static_assert(N >= 0 && N <= 15, "lgkmcnt range");
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void tie(bf16x8& v) { asm volatile("" : "+v"(v)); }

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>)
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

template <int NCO_, int NCI_, int TY_, int KW_ = 1, int TWN_ = 0, int CW_ = 1, int NSTG_ = 2, int RS_ = 0, int AR_ = 0>
struct WG {
    // AR = 1: the kernel-row form with the asm transposing reads (tr4_at) and counted waits, one
    // K group read ahead; AR = 2 the same without read-ahead — the same MFMAs in the same order
    // as AR = 0 (bit-identical)
    static constexpr int AR = AR_;
    static constexpr int NCO = NCO_, NCI = NCI_, TY = TY_;
    // row sweep (RS = 1): wave w owns kernel COLUMN dx = w % 3 and all three kernel rows, and walks
    // the stage's halo rows once: X row rho is read once and feeds the taps (dy, dx) of G rows
    // rho - dy, dy = 0..2 (the G fragments of the last three rows stay in registers).  Per 3 MFMAs
    // that is one X + one G fragment instead of one G + three X fragments per 3 MFMAs (the
    // default, wave = kernel row): the LDS read stream per MFMA halves.  Same operands, same
    // per-tap summation order (G rows ascending) -> bit-identical partials.
    static constexpr int RS = RS_;
    static_assert(!RS_ || (TWN_ == 0 && KW_ == 2), "row sweep: 3x3 taps, one column half per K-share wave");
    static_assert(!((RS_ & 2) && (RS_ & 8)), "per-row DMA pieces and loader waves exclude each other");
    // LDS stages in the pixel-tile ring: 2 (stage t+1 lands while stage t computes) or 3 (two
    // stages in flight: the weight-gradient loop had waited on its staging, PMC wait_any 0.48)
    static constexpr int NSTG = NSTG_;
    // CW waves per (kernel row, K-share) split the block's NCI ci tiles between them: the block
    // stages each pixel tile's G and X planes ONCE for all its ci tiles (CW = NCI: every 32-ci
    // tile of the layer in one block, so G is not re-staged per ci tile)
    static constexpr int CW = CW_, NCIW = NCI_ / CW_;
    // tap window: 0 = 3x3; 1 = taps {0,1}^2 (2 kernel rows, 2 columns: stride-2 phase convs)
    static constexpr int TWN = TWN_, TN = TWN_ ? 2 : 3;
    // KW waves per kernel row dy split each stage's K (pixel groups) between them;
    // their partial sums are added through LDS before the workspace store
    static constexpr int KW = KW_;
    // RS & 8: LW = 2 loader waves per block issue every LDS-DMA piece (the compute waves issue
    // none: their reads and MFMAs no longer queue behind ~7 DMA issues per stage)
    static constexpr int LW = (RS_ & 8) ? 2 : 0;
    static constexpr int WM = TN * KW * CW, NT = 64 * (WM + LW);
    static constexpr int SW = LW ? LW : WM;  // waves that stage
    static_assert(NCI % CW == 0, "ci tiles split evenly between the CW waves");
    static constexpr int CO_T = 32 * NCO, CI_T = 32 * NCI;
    static constexpr int GPL = 2 * NCO, XPL = 2 * NCI;         // 16-channel planes per stage
    static constexpr int XPIX = (TY + 2) * 34;                  // halo pixels per plane
    static constexpr int G_IPL = TY;                            // glds per G plane (one row each)
    static constexpr int X_IPL = (XPIX * 2 + 63) / 64;          // glds per X plane
    // plane strides = 128 (mod 256) bytes: the two 16-lane groups of a half-wave
    // read the same pixels of planes 2e and 2e+1 → disjoint bank halves.
    static constexpr int G_PLANE = G_IPL * 1024 + 128;
    static constexpr int X_PLANE = X_IPL * 1024 + 128;
    static constexpr int G_BYTES = GPL * G_PLANE;
    static constexpr int STAGE = G_BYTES + XPL * X_PLANE;
    static constexpr int G_INSTR = GPL * G_IPL, INSTR = G_INSTR + XPL * X_IPL;
    static constexpr int IPW = (INSTR + SW - 1) / SW;
    static constexpr int RED = CW * (KW - 1) * TN * 64 * (TN * NCO * NCIW * 16 + NCO) * 4;  // cross-wave K reduction
    static constexpr int LDS = NSTG * STAGE > RED ? NSTG * STAGE : RED;
    static_assert(LDS <= 163840, "LDS budget");
    static_assert((2 * TY) % KW == 0, "K groups split evenly between the KW waves of a row");
};

struct WgradArgs {
    isr_wgrad_desc d;
    float* ws;  // [splits][9*cout*cin (tap, co, ci) + cout (bias)]
    int splits, tiles;
};

// s_waitcnt vmcnt(n) for a run-time n in 0..15 (larger: 15 stays correct only as an upper
// bound of what may remain, so it waits for everything instead)
__device__ __forceinline__ void wait_vm_upto15(uint32_t n) {
#define ISR_W15(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n) {
        ISR_W15(1) ISR_W15(2) ISR_W15(3) ISR_W15(4) ISR_W15(5) ISR_W15(6) ISR_W15(7) ISR_W15(8)
        ISR_W15(9) ISR_W15(10) ISR_W15(11) ISR_W15(12) ISR_W15(13) ISR_W15(14) ISR_W15(15)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef ISR_W15
}

// One block's work: (ci tile, co tile, split) = the block index b within its conv.
template <class C>
__device__ __forceinline__ void wgrad_body(const isr_wgrad_desc& d, float* ws, int splits, int tiles, int b,
                                           int abl = 0) {
    // abl (tuning builds, timing probes, wrong results): 1 = no refill DMA after the first stage,
    // 2 = no MFMAs (the row sweep's reads stay)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int NCO = C::NCO, NCI = C::NCI, TY = C::TY;
    const int ncot = d.cout / C::CO_T, ncit = d.cin / C::CI_T;
    const int cit = b % ncit; b /= ncit;
    const int cot = b % ncot; b /= ncot;
    const int split = b;
    const int t0 = (int)((long)split * tiles / splits), t1 = (int)((long)(split + 1) * tiles / splits);
    const int wave = wave_id();
    const bool loader = C::LW && wave >= C::WM;                  // RS & 8: a DMA-only wave
    const bool stager = !C::LW || loader;
    const int sw = C::LW ? wave - C::WM : wave;                  // index among the staging waves
    const int dy = wave % C::TN, kh = (wave / C::TN) % C::KW;  // kernel row, K-share of this wave
    const int cw = wave / (C::TN * C::KW);                       // ci-tile group of this wave
    constexpr int NCIW = C::NCIW;
    const int lane = threadIdx.x & 63;
    const int nbx = d.wa / 32, nby = d.ha / TY;

    // ---- per-lane glds offsets relative to the tile bases (tile-invariant) --
    const size_t gps = plane_bytes(d.g), xps = plane_bytes(d.x);
    const int grow = d.g.wp * 32, xrow = d.x.wp * 32;
    const int cs4 = d.cout >> 2;
    uint32_t off[C::IPW];
#pragma unroll
    for (int k = 0; k < C::IPW; ++k) {
        const int j = sw + C::SW * k;
        uint32_t o = 0;
        if (j < C::G_INSTR) {
            const int pl = j / C::G_IPL, rr = j - pl * C::G_IPL;
            const int ch = cot * C::CO_T + pl * 16;
            if (d.g_sub2) {  // kernel channel ch = s*cout/4 + c  →  G pixel (2y + (s>>1), 2x + (s&1)), channel c
                const int sp = ch / cs4, c = ch - sp * cs4;
                o = (uint32_t)((size_t)(c >> 4) * gps + (size_t)(2 * rr + (sp >> 1)) * grow + (sp & 1) * 32 +
                               (lane >> 1) * 64 + (lane & 1) * 16);
            } else {
                o = (uint32_t)((size_t)(ch >> 4) * gps + (size_t)rr * grow + lane * 16);
            }
        } else if (j < C::INSTR) {
            const int jx = j - C::G_INSTR;
            const int pl = jx / C::X_IPL, jj = jx - pl * C::X_IPL;
            const int u = jj * 64 + lane;
            int q = u >> 1;
            if (q >= C::XPIX) q = 0;  // tail lanes of the last instruction: harmless duplicate
            const int row = q / 34, col = q - row * 34;
            if (d.x_sub2) {  // kernel channel c' = s*(cin/4) + c  →  x pixel (2row + (s>>1), 2col + (s&1)), channel c
                const int cpr = cit * C::CI_T + pl * 16, xs4 = d.cin >> 2;
                const int sp = cpr / xs4, c = cpr - sp * xs4;
                o = (uint32_t)((size_t)(c >> 4) * xps + (size_t)(2 * row + (sp >> 1)) * xrow + (2 * col + (sp & 1)) * 32 +
                               (u & 1) * 16);
            } else {
                o = (uint32_t)((size_t)((cit * C::CI_T) / 16 + pl) * xps + (size_t)row * xrow + col * 32 + (u & 1) * 16);
            }
        }
        off[k] = o;
    }
    auto lds_dst = [&](int j) -> int {
        if (j < C::G_INSTR) {
            const int pl = j / C::G_IPL, rr = j - pl * C::G_IPL;
            return pl * C::G_PLANE + rr * 1024;
        }
        const int jx = j - C::G_INSTR;
        const int pl = jx / C::X_IPL, jj = jx - pl * C::X_IPL;
        return C::G_BYTES + pl * C::X_PLANE + jj * 1024;
    };
    auto stage = [&](int t, int buf) {
        const int bx = t % nbx;
        int r = t / nbx;
        const int by = r % nby, img = r / nby;
        const int x0 = bx * 32, y0 = by * TY;
        // view_at with channel 0: the per-lane offsets carry the plane / sub-position
        const char* gb = d.g_sub2 ? view_at(d.g, img, 2 * y0, 2 * x0, 0) : view_at(d.g, img, y0, x0, 0);
        const char* xb = d.x_sub2 ? view_at(d.x, img, 2 * (y0 - 1), 2 * (x0 - 1), 0) : view_at(d.x, img, y0 - 1, x0 - 1, 0);
        char* dst = smem + buf * C::STAGE;
#pragma unroll
        for (int k = 0; k < C::IPW; ++k) {
            const int j = sw + C::SW * k;
            if (stager && j >= 0 && j < C::INSTR) glds16((j < C::G_INSTR ? gb : xb) + off[k], dst + lds_dst(j));
        }
    };

    f32x16 acc[C::TN][NCO][NCIW];
#pragma unroll
    for (int dx = 0; dx < C::TN; ++dx)
#pragma unroll
        for (int f = 0; f < NCO; ++f)
#pragma unroll
            for (int e = 0; e < NCIW; ++e)
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[dx][f][e][g] = 0.f;
    float bsum[NCO];
#pragma unroll
    for (int f = 0; f < NCO; ++f) bsum[f] = 0.f;
    const bool do_bias = d.db && cit == 0 && dy == 1 && cw == 0 && !loader;

    // transposed-read lane geometry: plane gi of the 32-channel fragment, pixel q + 8h, channels 4p..4p+3
    const int gi = (lane >> 4) & 1, hh = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
    const int a_lane = gi * C::G_PLANE + (8 * hh + q) * 32 + 8 * p;
    const int b_lane = C::G_BYTES + gi * C::X_PLANE + (8 * hh + q) * 32 + 8 * p;

    // this wave's copies per stage (wave-uniform)
    const int nps = (C::INSTR - sw + C::SW - 1) / C::SW < C::IPW ? (C::INSTR - sw + C::SW - 1) / C::SW : C::IPW;
    if (abl & 12) {
        // timing probe (tuning builds): half the blocks start ~half a stage later (4 = the second
        // 256 dispatched blocks, 8 = odd blocks), so co-resident blocks are not in phase
        const bool late = (abl & 4) ? ((blockIdx.x >> 8) & 1) : (blockIdx.x & 1);
        if (late)
            for (int i = 0; i < 56; ++i) __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int s0 = 0; s0 < C::NSTG - 1; ++s0)
        if (t0 + s0 < t1) stage(t0 + s0, s0);
    for (int t = t0; t < t1; ++t) {
        const int cur = (t - t0) % C::NSTG;
        if constexpr (C::NSTG == 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            // stage t landed; the younger stages already issued may stay in flight
            const int younger = t1 - 1 - t < C::NSTG - 2 ? t1 - 1 - t : C::NSTG - 2;
            wait_vm_upto15((uint32_t)(younger * nps));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (t + C::NSTG - 1 < t1 && !(abl & 1) && !(C::RS & 2)) stage(t + C::NSTG - 1, (t + C::NSTG - 1 - t0) % C::NSTG);
        if (loader) continue;  // RS & 8: the loader waves only stage
        const char* base = smem + cur * C::STAGE;
        if constexpr (C::RS) {
            // RS & 2: the next stage's LDS-DMA pieces go out one per halo row, between the row's
            // fragment reads and its MFMAs (issued as one block at the top of the stage they held
            // each wave's reads and MFMAs behind ~1,000 cycles of DMA issue); RS & 4: fragments
            // read two rows ahead instead of one
            const bool refill = t + C::NSTG - 1 < t1 && !(abl & 1);
            const char *rgb = nullptr, *rxb = nullptr;
            char* rdst = nullptr;
            if constexpr ((C::RS & 2) != 0) {
                const int tn = t + C::NSTG - 1;
                const int bx = tn % nbx;
                const int rq = tn / nbx;
                const int y0 = (rq % nby) * TY, img = rq / nby, x0 = bx * 32;
                rgb = d.g_sub2 ? view_at(d.g, img, 2 * y0, 2 * x0, 0) : view_at(d.g, img, y0, x0, 0);
                rxb = d.x_sub2 ? view_at(d.x, img, 2 * (y0 - 1), 2 * (x0 - 1), 0) : view_at(d.x, img, y0 - 1, x0 - 1, 0);
                rdst = smem + ((tn - t0) % C::NSTG) * C::STAGE;
            }
            auto piece = [&](auto K) {
                constexpr int k = decltype(K)::value;
                if constexpr ((C::RS & 2) != 0 && k < C::IPW) {
                    const int j = sw + C::SW * k;
                    if (refill && stager && j >= 0 && j < C::INSTR) glds16((j < C::G_INSTR ? rgb : rxb) + off[k], rdst + lds_dst(j));
                }
            };
            // wave (dx = dy-slot, column half kh): halo rows rho = 0..TY+1, G rows r = rho - tap row;
            // row rho+1's fragments are read while row rho's MFMAs run
            const int c0 = kh * 16, dxw = dy;
            const uint32_t ab = (uint32_t)(uintptr_t)ISR_LDS_PTR(base + a_lane + c0 * 32);
            const uint32_t bb =
                (uint32_t)(uintptr_t)ISR_LDS_PTR(base + b_lane + 2 * cw * NCIW * C::X_PLANE + (c0 + dxw) * 32);
            bf16x8 ga[TY][NCO];
            bf16x8 xb[TY + 2][NCIW];
            auto issue = [&](auto R) {
                constexpr int r = decltype(R)::value;
                if constexpr (r < TY)
                    sfor<NCO>([&](auto F) {
                        constexpr int o = 2 * decltype(F)::value * C::G_PLANE + r * 32 * 32;
                        ga[r][decltype(F)::value] = cat4(tr4_at<o>(ab), tr4_at<o + 4 * 32>(ab));
                    });
                sfor<NCIW>([&](auto E) {
                    constexpr int o = 2 * decltype(E)::value * C::X_PLANE + r * 34 * 32;
                    xb[r][decltype(E)::value] = cat4(tr4_at<o>(bb), tr4_at<o + 4 * 32>(bb));
                });
            };
            constexpr int AH = (C::RS & 4) ? 2 : 1;  // rows read ahead
            auto nrd = [](int r) constexpr { return r < TY + 2 ? 2 * NCIW + (r < TY ? 2 * NCO : 0) : 0; };
            issue(std::integral_constant<int, 0>{});
            if constexpr (AH == 2) issue(std::integral_constant<int, 1>{});
            sfor<TY + 2>([&](auto R) {
                constexpr int rho = decltype(R)::value;
                if constexpr (rho + AH < TY + 2) issue(std::integral_constant<int, rho + AH>{});
                piece(std::integral_constant<int, rho>{});
                // row rho's reads landed (the younger rows' may stay in flight)
                lgk_wait<nrd(rho + 1) + (AH == 2 ? nrd(rho + 2) : 0)>();
                if constexpr (rho < TY) {
#pragma unroll
                    for (int f = 0; f < NCO; ++f) tie(ga[rho][f]);
                    if (do_bias) {
#pragma unroll
                        for (int f = 0; f < NCO; ++f)
#pragma unroll
                            for (int e = 0; e < 8; ++e) bsum[f] += (float)ga[rho][f][e];
                    }
                }
#pragma unroll
                for (int e = 0; e < NCIW; ++e) tie(xb[rho][e]);
#pragma unroll
                for (int ty = 0; ty < 3; ++ty) {
                    const int r = rho - ty;
                    if (r < 0 || r >= TY || (abl & 2)) continue;
#pragma unroll
                    for (int f = 0; f < NCO; ++f)
#pragma unroll
                        for (int e = 0; e < NCIW; ++e) acc[ty][f][e] = mfma32(ga[r][f], xb[rho][e], acc[ty][f][e]);
                }
            });
            continue;
        }
        if constexpr (C::AR) {
            // K group kk: pixel row r = kk * KW / 2 + (kh >> 1) and column half (kh & 1) for even KW,
            // r = kk >> 1 and half kk & 1 for KW = 1; the run-time part goes into the base addresses
            constexpr int KW = C::KW, NK = 2 * TY / KW, TN = C::TN;
            const int rr = KW == 1 ? 0 : (kh >> 1), cr = KW == 1 ? 0 : (kh & 1) * 16;
            const uint32_t ab = (uint32_t)(uintptr_t)ISR_LDS_PTR(base + a_lane + (rr * 32 + cr) * 32);
            const uint32_t bb = (uint32_t)(uintptr_t)ISR_LDS_PTR(base + b_lane + 2 * cw * NCIW * C::X_PLANE +
                                                                  ((rr + dy) * 34 + cr) * 32);
            bf16x8 fa[NK][NCO];
            bf16x8 fb[NK][TN][NCIW];
            auto issue = [&](auto K) {
                constexpr int kk = decltype(K)::value;
                constexpr int rk = KW == 1 ? kk >> 1 : kk * KW / 2, ck = KW == 1 ? (kk & 1) * 16 : 0;
                sfor<NCO>([&](auto F) {
                    constexpr int o = 2 * decltype(F)::value * C::G_PLANE + (rk * 32 + ck) * 32;
                    fa[kk][decltype(F)::value] = cat4(tr4_at<o>(ab), tr4_at<o + 4 * 32>(ab));
                });
                sfor<TN>([&](auto D) {
                    sfor<NCIW>([&](auto E) {
                        constexpr int o = 2 * decltype(E)::value * C::X_PLANE + (rk * 34 + ck + decltype(D)::value) * 32;
                        fb[kk][decltype(D)::value][decltype(E)::value] = cat4(tr4_at<o>(bb), tr4_at<o + 4 * 32>(bb));
                    });
                });
            };
            constexpr int NR = 2 * NCO + 2 * TN * NCIW;  // reads per K group
            issue(std::integral_constant<int, 0>{});
            sfor<NK>([&](auto K) {
                constexpr int kk = decltype(K)::value;
                if constexpr (kk + 1 < NK && NR <= 15 && C::AR == 1) {
                    issue(std::integral_constant<int, kk + 1>{});
                    lgk_wait<NR>();
                } else if constexpr (C::AR == 1) {
                    lgk_wait<0>();
                    if constexpr (kk + 1 < NK) issue(std::integral_constant<int, kk + 1>{});
                } else {  // AR = 2: no read-ahead (one K group of fragments live: no spill at 64 x 96)
                    if constexpr (kk > 0) issue(std::integral_constant<int, kk>{});
                    lgk_wait<0>();
                }
#pragma unroll
                for (int f = 0; f < NCO; ++f) tie(fa[kk][f]);
#pragma unroll
                for (int dx = 0; dx < TN; ++dx)
#pragma unroll
                    for (int e = 0; e < NCIW; ++e) tie(fb[kk][dx][e]);
                if (do_bias) {
#pragma unroll
                    for (int f = 0; f < NCO; ++f)
#pragma unroll
                        for (int e = 0; e < 8; ++e) bsum[f] += (float)fa[kk][f][e];
                }
#pragma unroll
                for (int dx = 0; dx < TN; ++dx)
#pragma unroll
                    for (int f = 0; f < NCO; ++f)
#pragma unroll
                        for (int e = 0; e < NCIW; ++e) acc[dx][f][e] = mfma32(fa[kk][f], fb[kk][dx][e], acc[dx][f][e]);
            });
            continue;
        }
#pragma unroll
        for (int kk = 0; kk < 2 * TY / C::KW; ++kk) {
            const int kg = kk * C::KW + kh;
            const int r = kg >> 1, c0 = (kg & 1) * 16;
            bf16x8 fa[NCO];
#pragma unroll
            for (int f = 0; f < NCO; ++f) {
                const char* pa = base + a_lane + 2 * f * C::G_PLANE + (r * 32 + c0) * 32;
                fa[f] = cat4(lds_tr4(pa), lds_tr4(pa + 4 * 32));
            }
            if (do_bias) {
#pragma unroll
                for (int f = 0; f < NCO; ++f)
#pragma unroll
                    for (int e = 0; e < 8; ++e) bsum[f] += (float)fa[f][e];
            }
#pragma unroll
            for (int dx = 0; dx < C::TN; ++dx) {
                bf16x8 fb[NCIW];
#pragma unroll
                for (int e = 0; e < NCIW; ++e) {
                    const char* pb = base + b_lane + 2 * (cw * NCIW + e) * C::X_PLANE + ((r + dy) * 34 + c0 + dx) * 32;
                    fb[e] = cat4(lds_tr4(pb), lds_tr4(pb + 4 * 32));
                }
#pragma unroll
                for (int f = 0; f < NCO; ++f)
#pragma unroll
                    for (int e = 0; e < NCIW; ++e) acc[dx][f][e] = mfma32(fa[f], fb[e], acc[dx][f][e]);
            }
        }
    }

    if constexpr (C::KW > 1) {
        // add the K-shares of the KW waves of each kernel row (through the now idle stage LDS)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __syncthreads();
        constexpr int PER = C::TN * NCO * NCIW * 16 + NCO;  // floats per lane
        float* red = reinterpret_cast<float*>(smem);
        if (kh > 0 && !loader) {
            float* dst = red + ((size_t)((cw * (C::KW - 1) + kh - 1) * C::TN + dy) * 64 + lane) * PER;
            int q = 0;
#pragma unroll
            for (int dx = 0; dx < C::TN; ++dx)
#pragma unroll
                for (int f = 0; f < NCO; ++f)
#pragma unroll
                    for (int e = 0; e < NCIW; ++e)
#pragma unroll
                        for (int g = 0; g < 16; ++g) dst[q++] = acc[dx][f][e][g];
#pragma unroll
            for (int f = 0; f < NCO; ++f) dst[q++] = bsum[f];
        }
        __syncthreads();
        if (kh > 0 || loader) return;
#pragma unroll
        for (int k = 1; k < C::KW; ++k) {
            const float* src = red + ((size_t)((cw * (C::KW - 1) + k - 1) * C::TN + dy) * 64 + lane) * PER;
            int q = 0;
#pragma unroll
            for (int dx = 0; dx < C::TN; ++dx)
#pragma unroll
                for (int f = 0; f < NCO; ++f)
#pragma unroll
                    for (int e = 0; e < NCIW; ++e)
#pragma unroll
                        for (int g = 0; g < 16; ++g) acc[dx][f][e][g] += src[q++];
#pragma unroll
            for (int f = 0; f < NCO; ++f) bsum[f] += src[q++];
        }
    }

    if (loader) return;  // (KW == 1 forms: the loader waves leave after the loop)
    // ---- partial sums: ws[split][tap][co][ci], D[co = (g&3)+8(g>>2)+4h][ci = l31]
    const int l31 = lane & 31;
    float* wsp = ws + (size_t)split * (9 * d.cout * d.cin + d.cout);
#pragma unroll
    for (int dx = 0; dx < C::TN; ++dx) {
        // accumulator slot dx = kernel column (default) or kernel row (row sweep; dy = the column)
        float* wt = wsp + (size_t)(C::RS ? dx * 3 + dy : dy * 3 + dx) * d.cout * d.cin;
#pragma unroll
        for (int f = 0; f < NCO; ++f)
#pragma unroll
            for (int e = 0; e < NCIW; ++e)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int co = cot * C::CO_T + f * 32 + (g & 3) + 8 * (g >> 2) + 4 * hh;
                    const int ci = cit * C::CI_T + (cw * NCIW + e) * 32 + l31;
                    wt[(size_t)co * d.cin + ci] = acc[dx][f][e][g];
                }
    }
    if (d.db && cit == 0 && dy == 1 && cw == 0) {
        float* bp = wsp + (size_t)9 * d.cout * d.cin;
#pragma unroll
        for (int f = 0; f < NCO; ++f) {
            const float v = bsum[f] + __shfl_xor(bsum[f], 32);
            if (hh == 0) bp[cot * C::CO_T + f * 32 + (gi * 16 + (lane & 15))] = v;
        }
    }
}

template <class C>
__global__ __launch_bounds__(C::NT) void wgrad3x3_kernel(WgradArgs a) {
    wgrad_body<C>(a.d, a.ws, a.splits, a.tiles, xcd_remap(blockIdx.x, gridDim.x));
}

// Several weight gradients over the same pixel grid in ONE launch (the 5 convs of an RDB read
// one dense buffer and one gradient buffer): the blocks of conv t are [start[t], start[t+1]),
// each conv's partials in its own workspace range.  With all the convs' (co, ci) tile pairs in
// one grid, a split count ~5x smaller fills the chip — each block walks ~5x more pixel tiles and
// the split-K partials written and reduced shrink by the same factor.
constexpr int WG_GROUP_MAX = 5;
struct WgradGroupArgs {
    isr_wgrad_desc d[WG_GROUP_MAX];
    float* ws[WG_GROUP_MAX];
    int start[WG_GROUP_MAX + 1];   // wgrad blocks
    int rstart[WG_GROUP_MAX + 1];  // reduce blocks
    int pstart[WG_GROUP_MAX + 1];  // (co, ci) tile pairs
    int n, splits, tiles, pairs;
    int order;  // block order: 0 = member-major, 1 = split-major over all members' tile pairs
    int abl;    // timing-probe ablations (tuning builds; 0 in production)
};

__device__ __forceinline__ int group_member(const WgradGroupArgs& g, const int* start, int b) {
    int t = 0;
#pragma unroll
    for (int k = 1; k < WG_GROUP_MAX; ++k) t += (k < g.n && b >= start[k]) ? 1 : 0;
    return t;
}

// Block order.  Member-major (0): conv t's blocks (ci tile, co tile, split) in turn, so an XCD's
// contiguous share of the grid (xcd_remap) holds one or two members and each member re-reads the
// dense buffer's channels it shares with the others.  Split-major (1): the blocks of one split —
// one pixel range — over ALL members' tile pairs are adjacent, so the 26 blocks that read the same
// pixel rows of the dense and gradient buffers run together on one XCD and share its L2.
template <class C>
__global__ __launch_bounds__(C::NT) void wgrad3x3_group_kernel(WgradGroupArgs g) {
    const int l = xcd_remap(blockIdx.x, gridDim.x);
    int t, b;
    if (g.order == 1) {
        const int split = l / g.pairs, p = l - split * g.pairs;
        t = group_member(g, g.pstart, p);
        b = (p - g.pstart[t]) + (g.pstart[t + 1] - g.pstart[t]) * split;
    } else {
        t = group_member(g, g.start, l);
        b = l - g.start[t];
    }
#ifdef ISR_TUNING
    wgrad_body<C>(g.d[t], g.ws[t], g.splits, g.tiles, b, g.abl);
#else
    wgrad_body<C>(g.d[t], g.ws[t], g.splits, g.tiles, b);
#endif
}

// dW[co][ci][tap] (reference OIHW) = scale * sum_s ws[s][tap][co'][ci];  co' = kernel channel order.
// One block per (co', 32-ci run): 4 split-slices x 32 ci threads each sum 9 tap rows
// (coalesced 128-B reads per tap), the slices are added through LDS, and the block writes its
// 32 x 9 outputs as ONE contiguous run of dW — the transposing scatter of the column-wise
// reduce below (4-B stores 36 B apart) took 0.5 ms per call on the discriminator's 512 x 2048
// phase-expanded weight.  Requires cin % 32 == 0.
__global__ __launch_bounds__(128) void wgrad_reduce_t_kernel(WgradArgs a) {
    __shared__ float red[4][9][33];
    const isr_wgrad_desc& d = a.d;
    const size_t per = (size_t)9 * d.cout * d.cin;
    const size_t row = per + d.cout;
    const int ncb = d.cin / 32;
    const int cok = blockIdx.x / ncb, ci0 = (blockIdx.x - cok * ncb) * 32;
    const int c = threadIdx.x & 31, slice = threadIdx.x >> 5;
    float acc[9], bacc = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = 0.f;
    const float* src = a.ws + (size_t)cok * d.cin + ci0 + c;
    const bool bias_blk = d.db && ci0 == 0;
    for (int sp = slice; sp < a.splits; sp += 4) {
        const float* r = src + (size_t)sp * row;
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] += r[(size_t)t * d.cout * d.cin];
        if (bias_blk && c == 0) bacc += a.ws[(size_t)sp * row + per + cok];
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) red[slice][t][c] = acc[t];
    if (bias_blk && c == 0) red[slice][0][32] = bacc;
    __syncthreads();
    const int cs4 = d.cout >> 2;
    const int co = d.g_sub2 ? (cok % cs4) * 4 + cok / cs4 : cok;
    float* dst = d.dw + ((size_t)co * d.cin + ci0) * 9;
    for (int o = threadIdx.x; o < 32 * 9; o += 128) {
        const int cc = o / 9, t = o - cc * 9;
        dst[o] = (red[0][t][cc] + red[1][t][cc] + red[2][t][cc] + red[3][t][cc]) * d.scale;
    }
    if (bias_blk && threadIdx.x == 0) d.db[co] = (red[0][0][32] + red[1][0][32] + red[2][0][32] + red[3][0][32]) * d.scale;
}

// Workspace rows are [splits][9*cout*cin + cout] (the bias partials follow each
// split's dW partials).  Block = 16 split-slices x 16 float4 columns: every thread streams
// S/16 rows of one 16-byte column, the 16 slices are summed through LDS in slice order.  (The
// first form, 4 slices x 64 columns, launched 181 blocks for a growth conv's 46 K weights —
// under one per CU — and each thread walked S/4 = 16..64 dependent rows: ~20 us per reduce,
// latency-bound, on the side stream beside the RDB gather convs.)
// RED_SL split-slices x RED_COLS 16-byte columns per 256-thread block: every thread streams
// S / RED_SL rows of one column with all its loads in flight (UNR-deep unroll), the slices are
// summed through LDS in slice order.  Production <16, 16, 4>; the tuning build picks others
// with ISR_WGRAD_RED (timing A/B of the cfg3 step).
template <int RED_SL, int RED_COLS, int UNR>
__device__ __forceinline__ void wgrad_reduce_body(const isr_wgrad_desc& d, const float* ws, int splits, int blk) {
    static_assert(RED_SL * RED_COLS == 256, "one 256-thread block");
    __shared__ f32x4 red[RED_SL][RED_COLS];
    const size_t per = (size_t)9 * d.cout * d.cin;
    const size_t row = per + d.cout;
    const int nv = (int)(row / 4);
    const int lc = threadIdx.x % RED_COLS, slice = threadIdx.x / RED_COLS;
    const int col = blk * RED_COLS + lc;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (col < nv) {
        const f32x4* src = reinterpret_cast<const f32x4*>(ws) + col;
#pragma unroll UNR
        for (int sp = slice; sp < splits; sp += RED_SL) acc += src[(size_t)sp * (row / 4)];
    }
    red[slice][lc] = acc;
    __syncthreads();
    if (slice != 0 || col >= nv) return;
    acc = red[0][lc];
#pragma unroll
    for (int k = 1; k < RED_SL; ++k) acc += red[k][lc];
    const int cs4 = d.cout >> 2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const size_t idx = (size_t)col * 4 + e;
        if (idx < per) {
            const int ci = (int)(idx % d.cin);
            const int cok = (int)((idx / d.cin) % d.cout);
            const int tap = (int)(idx / ((size_t)d.cin * d.cout));
            const int co = d.g_sub2 ? (cok % cs4) * 4 + cok / cs4 : cok;
            d.dw[((size_t)co * d.cin + ci) * 9 + tap] = acc[e] * d.scale;
        } else if (d.db) {
            const int cok = (int)(idx - per);
            const int co = d.g_sub2 ? (cok % cs4) * 4 + cok / cs4 : cok;
            d.db[co] = acc[e] * d.scale;
        }
    }
}

template <int RED_SL, int RED_COLS, int UNR>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(WgradArgs a) {
    wgrad_reduce_body<RED_SL, RED_COLS, UNR>(a.d, a.ws, a.splits, blockIdx.x);
}

__global__ __launch_bounds__(256) void wgrad_reduce_group_kernel(WgradGroupArgs g) {
    const int b = blockIdx.x;
    const int t = group_member(g, g.rstart, b);
    wgrad_reduce_body<16, 16, 4>(g.d[t], g.ws[t], g.splits, b - g.rstart[t]);
}

template <int SL, int COLS, int UNR>
static void launch_reduce(const WgradArgs& a, hipStream_t s) {
    const size_t nv = ((size_t)9 * a.d.cout * a.d.cin + a.d.cout) / 4;
    hipLaunchKernelGGL((wgrad_reduce_kernel<SL, COLS, UNR>), dim3((unsigned)((nv + COLS - 1) / COLS)), dim3(256), 0, s,
                       a);
}

// Variants (isr_wgrad3x3_variant; tools/tune_wgrad.py).  TY = pixel rows per
// stage: a longer stage gives each barrier more MFMAs and halves the X halo
// overhead ((TY+2)/TY), at the price of LDS (2 blocks/CU need <= 80 KB).
template <int TY, int KW = 1>
struct Fam {
    using C22 = WG<2, 2, TY, KW>;
    using C12 = WG<1, 2, TY, KW>;
    using C21 = WG<2, 1, TY, KW>;
    using C11 = WG<1, 1, TY, KW>;
};

static int wgrad_splits(const isr_wgrad_desc* d, int tiles, int pairs, int target, int min_splits = 1) {
    if (d->splits > 0) return d->splits < tiles ? d->splits : tiles;
    int s = (target + pairs - 1) / pairs;
    if (s < min_splits) s = min_splits;
    return s < tiles ? s : tiles;
}

template <class C>
static void wgrad_geometry(const isr_wgrad_desc* d, int* tiles, int* splits) {
    *tiles = d->n * (d->ha / C::TY) * (d->wa / 32);
    // ~640 blocks of <= 6 waves; blocks with more K-share waves need proportionally fewer
    // splits (each split-K partial costs a workspace write + reduce read)
    // CW > 1 (all of a layer's ci tiles in one block, up to 15 waves): ~2 blocks per CU slot.
    // KW == 2 (8-row stages): ~512 blocks and >= 64 splits — the split-K sweep
    // (tools/tune_wgrad.py --splits, profiles/r02_wgrad_splits.jsonl) put the best split count
    // at 128-256 for 2-4 (co, ci) tile pairs and at 64 for 12-16 pairs: 6-20 % under the
    // earlier ~640-block target, whose extra partials cost more in the reduce than they gain
    const int target = C::CW > 1 ? (C::LDS > 81920 ? 512 : 1024) / (C::CO_T == 64 && d->cin > C::CI_T ? 2 : 1)
                                 : (C::KW > 2 ? 640 * 2 / C::KW : (C::KW == 2 ? 512 : 640));
    // (the 64-split floor only for the generator's few-pair shapes: the discriminator's wide
    // layers have 64..1024 pairs, where it would multiply the partials — 2.4 GB at 512 x 2048)
    const int pairs = (d->cout / C::CO_T) * (d->cin / C::CI_T);
    *splits = wgrad_splits(d, *tiles, pairs, target, C::KW == 2 && pairs <= 16 ? 64 : 1);
}

// parts: 1 = the split-K partials, 2 = their reduction into dW / db, 3 = both (in stream order)
template <class C>
static int launch_wgrad(const isr_wgrad_desc* d, void* ws, size_t ws_bytes, hipStream_t s, int parts = 3) {
    if (d->ha % C::TY || d->cout % C::CO_T || d->cin % C::CI_T) return -2;
    WgradArgs a;
    a.d = *d;
    wgrad_geometry<C>(d, &a.tiles, &a.splits);
    if (ws_bytes < ((size_t)a.splits * 9 * d->cout * d->cin + (size_t)a.splits * d->cout) * 4) return -3;
    a.ws = (float*)ws;
#ifdef ISR_TUNING
    // timing probes of the training step (outputs wrong): no weight gradients at all / no reduce
    static const bool skip_all = getenv("ISR_WGRAD_SKIP") != nullptr, skip_red = getenv("ISR_WGRAD_NO_REDUCE") != nullptr;
    if (skip_all) return 0;
#endif
    if (parts & 1) {
        auto kern = wgrad3x3_kernel<C>;
        lds_limit((const void*)kern, C::LDS);
        const int blocks = a.splits * (d->cout / C::CO_T) * (d->cin / C::CI_T);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(C::NT), C::LDS, s, a);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (!(parts & 2)) return 0;
#ifdef ISR_TUNING
    if (skip_red) return 0;
#endif
    // the transposing reduce has one block per (co, 32 ci): it pays only for large weights (the
    // discriminator's phase-expanded 128..512 x 512..2048); the generator's <= 256 x 192 keep
    // the column-wise reduce (more blocks: 30 vs 48 us per wgrad at 32 x 64)
    if (d->cin % 32 == 0 && (size_t)d->cout * d->cin >= 65536) {
        hipLaunchKernelGGL(wgrad_reduce_t_kernel, dim3((unsigned)(d->cout * (d->cin / 32))), dim3(128), 0, s, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
#ifdef ISR_TUNING
    static const int red_v = getenv("ISR_WGRAD_RED") ? atoi(getenv("ISR_WGRAD_RED")) : 0;
    switch (red_v) {
        case 1: launch_reduce<32, 8, 8>(a, s); return hipGetLastError() == hipSuccess ? 0 : -1;
        case 2: launch_reduce<8, 32, 8>(a, s); return hipGetLastError() == hipSuccess ? 0 : -1;
        case 3: launch_reduce<16, 16, 8>(a, s); return hipGetLastError() == hipSuccess ? 0 : -1;
        case 4: launch_reduce<64, 4, 4>(a, s); return hipGetLastError() == hipSuccess ? 0 : -1;
        default: break;
    }
#endif
    launch_reduce<16, 16, 4>(a, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <class Fm, class F>
static auto pick_in(const isr_wgrad_desc* d, bool co1, F&& f) {
    const bool co2 = !co1 && d->cout % 64 == 0, ci2 = d->cin % 64 == 0;
    if (co2 && ci2) return f(typename Fm::C22());
    if (ci2) return f(typename Fm::C12());
    if (co2) return f(typename Fm::C21());
    return f(typename Fm::C11());
}

// ci-split forms (WG CW > 1): every ci tile of the layer (or half of them at cout 64 / cin 192)
// in one block, so each pixel tile's G and X planes are staged once per block
template <int TY, class F>
static auto pick_cw(const isr_wgrad_desc* d, F&& f, bool* ok) {
    *ok = true;
    if (d->taps == 0 && !d->x_sub2) {
        if (d->cout % 64 != 0) {  // cout 32 (growth convs)
            switch (d->cin) {
                case 64: return f(WG<1, 2, TY, 1, 0, 2>());
                case 96: return f(WG<1, 3, 4, 1, 0, 3>());
                case 128: return f(WG<1, 4, 4, 1, 0, 4>());
                case 160: return f(WG<1, 5, 4, 1, 0, 5>());
                default: break;
            }
        } else if (d->cin == 192) {
            return f(WG<2, 3, 4, 1, 0, 3>());
        } else if (d->cin % 64 == 0) {
            return f(WG<2, 2, TY, 1, 0, 2>());
        }
    }
    *ok = false;
    return f(Fam<4>::C11());
}

// AR = 1 (production): the asm-read forms (WG::AR / WG::RS); 0 = compiler-visible LDS reads;
// the 64 x 96 final-conv tile reads without read-ahead (AR 2: 8 B of scratch with it)
template <int AR, class F>
static auto pick_default(const isr_wgrad_desc* d, F&& f) {
    // the discriminator's wide layers (variant 14: -0.5 % per SRGAN step, same-box A/B): 64 co x
    // 128 (or 64) ci per block, 8-12 waves splitting the ci tiles, each pixel tile staged once
    if (d->cout % 64 == 0 && d->ha % 4 == 0 && !d->g_sub2) {
        if (d->taps == 1 && d->cin % 128 == 0) return f(WG<2, 4, 4, 1, 1, 4, 2, 0, AR>());
        if (d->taps == 0 && d->cout >= 128 && d->cin % 128 == 0) return f(WG<2, 4, 4, 1, 0, 4, 2, 0, AR>());
        if (d->taps == 0 && d->cout >= 128 && d->cin % 64 == 0) return f(WG<2, 2, 4, 1, 0, 2, 2, 0, AR>());
    }
    if (d->taps == 1) return f(WG<1, 1, 8, 2, 1, 1, 2, 0, AR>());  // stride-2 phase conv: taps {0,1}^2, 4 waves
    // production (tools/tune_wgrad.py, MI355X, N=16 128²): 32x32 (co, ci) tiles; 4-row
    // stages when cin % 64 == 32 (96, 160), else 8-row stages with 2 waves per kernel
    // row (variant 5): 4-11 % under the round-1 choice (16-row stages, 4 waves per
    // row) on cin 64 / 128 / 192 and the sub2 Scaler shape, on two boxes
    // the RDB final conv (cin 192, cout 64): 64x96 (co, ci) per block, 9 waves splitting the
    // ci tiles (each pixel tile staged once per block): 81-86 vs 98-104 us
    if (d->cin == 192 && d->cout == 64 && !d->g_sub2 && !d->x_sub2 && d->ha % 4 == 0)
        return f(WG<2, 3, 4, 1, 0, 3, 2, 0, AR ? 2 : 0>());
    if (d->cin % 64 == 32) return f(WG<1, 1, 4, 1, 0, 1, 2, 0, AR>());
    // 8-row stages, 2 waves per kernel row; with AR as the row sweep (WG::RS, same bits)
    if (d->ha % 8 == 0) return f(WG<1, 1, 8, 2, 0, 1, 2, AR, 0>());
    if (d->ha % 4 == 0) return f(WG<1, 1, 4, 1, 0, 1, 2, 0, AR>());
    return f(WG<1, 1, 2, 1, 0, 1, 2, 0, AR>());
}

// variant 0: the production pick; 16: the same tiles and split counts with compiler-visible LDS
// reads (pick_default<0>: the reference the asm-read / row-sweep forms must equal bit for bit,
// tests/test_gpu_kernels.py); 1-15: earlier tile forms, tuning builds only (-DISR_TUNING)
template <class F>
static auto wgrad_pick(const isr_wgrad_desc* d, int variant, F&& f) {
    if (variant == 16) return pick_default<0>(d, f);
#ifdef ISR_TUNING
    switch (variant) {
        case 14: {  // ci-split forms for the discriminator's wide layers (64 co x 128 ci per block)
            if (d->cout % 64 == 0 && d->ha % 4 == 0) {
                if (d->taps == 1 && d->cin % 128 == 0) return f(WG<2, 4, 4, 1, 1, 4>());
                if (d->taps == 0 && d->cin % 128 == 0 && !d->g_sub2) return f(WG<2, 4, 4, 1, 0, 4>());
                if (d->taps == 0 && d->cin % 64 == 0 && !d->g_sub2) return f(WG<2, 2, 4, 1, 0, 2>());
            }
            break;
        }
        case 12:
        case 13: {
            bool ok;
            auto r = variant == 12 ? pick_cw<4>(d, f, &ok) : pick_cw<8>(d, f, &ok);
            if (ok) return r;
            break;
        }
        case 1: return pick_in<Fam<2>>(d, false, f);  // round-1 production: 2-row stages
        case 2: return pick_in<Fam<4>>(d, false, f);  // 4-row stages (C22: 92 KB LDS, 1 block/CU)
        case 3: return pick_in<Fam<4>>(d, true, f);   // 4-row stages, 32-cout tiles (<= 75 KB)
        case 4: return f(Fam<8>::C11());              // 8-row stages, 32x32 tiles
        case 5: return f(Fam<8, 2>::C11());           // variant 4 with 2 waves per kernel row (K split)
        case 6: return f(Fam<4, 2>::C11());           // 4-row stages, 2 waves per kernel row
        case 7: return f(Fam<8, 2>::C12());           // 32x64 tiles, 2 waves per kernel row
        case 8: return f(Fam<8, 4>::C11());           // 4 waves per kernel row (12 per block), half the splits
        case 9: return f(Fam<16, 4>::C11());          // 16-row stages, 4 waves per kernel row
        case 10: return f(Fam<4, 4>::C11());          // 4-row stages, 4 waves per kernel row
        case 11: return f(Fam<16, 2>::C11());         // 16-row stages, 2 waves per kernel row
        case 15:                                      // variant 5 as a row sweep (WG::RS)
            if (d->taps == 0 && d->ha % 8 == 0) return f(WG<1, 1, 8, 2, 0, 1, 2, 1>());
            break;
        default: break;
    }
    // A/B of the kernel-row forms with compiler-visible LDS reads (tuning builds: ISR_WGRAD_AR=0)
    static const bool ar = !getenv("ISR_WGRAD_AR") || atoi(getenv("ISR_WGRAD_AR")) != 0;
    if (!ar) return pick_default<0>(d, f);
#endif
    return pick_default<1>(d, f);
}

size_t wgrad3x3_workspace_bytes(const isr_wgrad_desc* d, int variant) {
    return wgrad_pick(d, variant, [&](auto c) {
        using C = decltype(c);
        int tiles, splits;
        wgrad_geometry<C>(d, &tiles, &splits);
        return ((size_t)splits * 9 * d->cout * d->cin + (size_t)splits * d->cout) * 4;
    });
}

int wgrad3x3_dispatch(const isr_wgrad_desc* d, int variant, void* ws, size_t ws_bytes, hipStream_t s, int parts) {
    return wgrad_pick(d, variant, [&](auto c) { return launch_wgrad<decltype(c)>(d, ws, ws_bytes, s, parts); });
}

// ---- grouped weight gradients (isr_wgrad3x3_group) ----
// every member: plain 3x3 (no sub2 / tap window), cout % 32 == cin % 32 == 0, the same n / ha /
// wa; 32x32 (co, ci) tiles, 8-row stages with 2 waves per kernel row (4-row stages when ha % 8)
template <class C>
static int group_plan(const isr_wgrad_desc* ds, int n, WgradGroupArgs* g, size_t* bytes) {
    if (n < 1 || n > WG_GROUP_MAX) return -2;
    int pairs = 0;
    for (int t = 0; t < n; ++t) {
        const isr_wgrad_desc& d = ds[t];
        if (d.g_sub2 || d.x_sub2 || d.taps || d.cout % C::CO_T || d.cin % C::CI_T || d.ha % C::TY || d.n != ds[0].n ||
            d.ha != ds[0].ha || d.wa != ds[0].wa)
            return -2;
        pairs += (d.cout / C::CO_T) * (d.cin / C::CI_T);
    }
    const int tiles = ds[0].n * (ds[0].ha / C::TY) * (ds[0].wa / 32);
    // ~1024 blocks: the cfg3 step is flat from 28 to 56 splits over an RDB's 26 tile pairs and
    // loses 0.4 ms at 20, 1.7 ms at 8 (tuning sweep, profiles/r04_wgrad_group_splits.jsonl)
    int splits = (1024 + pairs - 1) / pairs;
#ifdef ISR_TUNING
    if (const char* e = getenv("ISR_WGRAD_GROUP_SPLITS")) splits = atoi(e);  // split sweep (tuning builds)
#endif
    if (splits < 1) splits = 1;
    if (splits > tiles) splits = tiles;
    size_t off = 0;
    int blk = 0, rblk = 0;
    for (int t = 0; t < n; ++t) {
        const isr_wgrad_desc& d = ds[t];
        g->d[t] = d;
        g->ws[t] = (float*)(uintptr_t)off;  // byte offset for now; based on the workspace below
        off += ((size_t)splits * 9 * d.cout * d.cin + (size_t)splits * d.cout) * 4;
        off = (off + 255) / 256 * 256;
        g->start[t] = blk;
        g->pstart[t] = blk / splits;
        blk += splits * (d.cout / C::CO_T) * (d.cin / C::CI_T);
        g->rstart[t] = rblk;
        rblk += (int)((((size_t)9 * d.cout * d.cin + d.cout) / 4 + 15) / 16);
    }
    g->start[n] = blk;
    g->rstart[n] = rblk;
    g->pstart[n] = pairs;
    for (int t = n + 1; t <= WG_GROUP_MAX; ++t) g->start[t] = g->rstart[t] = g->pstart[t] = 0x7fffffff;
    g->n = n;
    g->splits = splits;
    g->tiles = tiles;
    g->pairs = pairs;
    // block order: split-major (1) in production; the pair-major A/B form (0) only in tuning
    // builds (both give the same bits: every block's partial and the reduce are unchanged)
    g->order = 1;
    g->abl = 0;
#ifdef ISR_TUNING
    static const int abl_probe = getenv("ISR_WGRAD_ABLATE") ? atoi(getenv("ISR_WGRAD_ABLATE")) : 0;
    g->abl = abl_probe;
    static const int order_probe = getenv("ISR_WGRAD_GROUP_ORDER") ? atoi(getenv("ISR_WGRAD_GROUP_ORDER")) : 1;
    g->order = order_probe;
#endif
    *bytes = off;
    return 0;
}

// variant 0: production (the row sweep, or the asm-read 4-row form); 1: the same tiles and split
// counts with compiler-visible LDS reads (bit-identical reference, tests/test_gpu_kernels.py)
template <class F>
static auto group_pick(const isr_wgrad_desc* ds, int n, F&& f, int variant = 0) {
    bool ty8 = true, ty16 = true;
    for (int t = 0; t < n; ++t) {
        ty8 = ty8 && ds[t].ha % 8 == 0;
        ty16 = ty16 && ds[t].ha % 16 == 0;
    }
#ifdef ISR_TUNING
    // tile-config probe of the grouped launch (tuning builds): 1 = 4-row stages, 1 wave per row;
    // 2 = 8-row stages, 4 waves per row; 3 = 16-row stages, 2 waves per row; 4 = 8-row, 1 wave
    static const int cfg = getenv("ISR_WGRAD_GROUP_CFG") ? atoi(getenv("ISR_WGRAD_GROUP_CFG")) : 0;
    if (cfg == 1) return f(Fam<4>::C11());
    if (cfg == 2 && ty8) return f(Fam<8, 4>::C11());
    if (cfg == 3 && ty16) return f(Fam<16, 2>::C11());
    if (cfg == 4 && ty8) return f(Fam<8>::C11());
    if (cfg == 5) return f(WG<1, 1, 4, 1, 0, 1, 3>());          // 4-row stages, 3-stage ring
    if (cfg == 6) return f(WG<1, 1, 4, 2, 0, 1, 3>());          // 4-row stages, 2 waves per row, 3 stages
    if (cfg == 7 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 3>());   // production tile, 3 stages (1 block / CU)
    if (cfg == 8 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 1>());   // production tile, row sweep
    if (cfg == 9 && ty16) return f(WG<1, 1, 16, 2, 0, 1, 2, 1>()); // 16-row stages, row sweep (1 block / CU)
    if (cfg == 10 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 3, 1>());  // row sweep, 3 stages
    if (cfg == 11 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 0, 1>());  // kernel-row form, asm reads
    if (cfg == 12) return ty8 ? f(Fam<8, 2>::C11()) : f(Fam<4>::C11());  // round-4 production
    if (cfg == 13 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 3>());  // row sweep + DMA one piece per row
    if (cfg == 14 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 5>());  // row sweep, 2 rows read ahead
    if (cfg == 15 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 7>());  // both
    if (cfg == 16 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 9>());  // row sweep + 2 loader waves
    if (cfg == 17 && ty8) return f(WG<1, 1, 8, 2, 0, 1, 2, 13>()); // + 2 rows read ahead
#endif
    (void)ty16;
    if (variant == 1) return ty8 ? f(WG<1, 1, 8, 2, 0, 1, 2, 0, 0>()) : f(WG<1, 1, 4, 1, 0, 1, 2, 0, 0>());
    // 8-row stages, 2 waves per kernel column: the row sweep (WG::RS)
    return ty8 ? f(WG<1, 1, 8, 2, 0, 1, 2, 1>()) : f(WG<1, 1, 4, 1, 0, 1, 2, 0, 1>());
}

size_t wgrad3x3_group_workspace_bytes(const isr_wgrad_desc* ds, int n, int variant) {
    return group_pick(ds, n, [&](auto c) -> size_t {
        WgradGroupArgs g;
        size_t bytes = 0;
        return group_plan<decltype(c)>(ds, n, &g, &bytes) == 0 ? bytes : 0;
    }, variant);
}

int wgrad3x3_group_dispatch(const isr_wgrad_desc* ds, int n, void* ws, size_t ws_bytes, hipStream_t s, int variant) {
    return group_pick(ds, n, [&](auto c) -> int {
        using C = decltype(c);
        WgradGroupArgs g;
        size_t bytes = 0;
        const int rc = group_plan<C>(ds, n, &g, &bytes);
        if (rc) return rc;
        if (ws_bytes < bytes) return -3;
        for (int t = 0; t < n; ++t) g.ws[t] = (float*)((char*)ws + (uintptr_t)g.ws[t]);
        auto kern = wgrad3x3_group_kernel<C>;
        lds_limit((const void*)kern, C::LDS);
        hipLaunchKernelGGL(kern, dim3(g.start[n]), dim3(C::NT), C::LDS, s, g);
        if (hipGetLastError() != hipSuccess) return -1;
        hipLaunchKernelGGL(wgrad_reduce_group_kernel, dim3(g.rstart[n]), dim3(256), 0, s, g);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }, variant);
}

}  // namespace isr
