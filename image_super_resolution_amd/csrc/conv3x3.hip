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
#include <string.h>

#include "isr_common.h"

namespace isr {

// Timing stamps (tuning builds only, isr_tuning_conv_stamps): per block, wall-clock
// (s_memrealtime, 100 MHz) at entry / first chunk landed / main loop done / epilogue
// done, plus the raw HW_ID and XCC_ID registers.  Written by a vector store of lane 0
// of wave 0 into a buffer of its own (never read by the kernel).
#ifdef ISR_TUNING
__device__ unsigned long long* g_conv_stamps;
#endif
__device__ __forceinline__ void conv_stamp(int slot, int row = -1) {
#ifdef ISR_TUNING
    unsigned long long* p = g_conv_stamps;
    if (p != nullptr && threadIdx.x == 0 && row != -2) {
        unsigned long long t;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");  // not hoistable
        p[(size_t)(row < 0 ? blockIdx.x : row) * 8 + slot + threadIdx.x] = t;
        if (slot == 0 && row < 0) {
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); // HW_REG_XCC_ID
            p[(size_t)blockIdx.x * 8 + 6 + threadIdx.x] = hw;
            p[(size_t)blockIdx.x * 8 + 7 + threadIdx.x] = xcc;
        }
    }
#else
    (void)slot;
    (void)row;
#endif
}

template <int R_, int WM_, int NF_, int KC_, int NST_, int CIN_ = 0, int ABL_ = 0, int PIPE_ = (NF_ == 1), int EPQ_ = 4,
          int SPL_ = 0, int TWN_ = 0, int NSW_ = 0, int FOLD_ = 0, int H_ = 0>
struct C3 {
    static constexpr int R = R_, WM = WM_, NF = NF_, KC = KC_, NST = NST_;
    // storage type of activations and weights: 0 = bf16, 1 = fp16 (isr_conv_desc.f16, inference)
    static constexpr bool H = H_ != 0;
    // 1: the RDB residual fold (r1 == the conv's own input channels, see fold_ok) is compiled in;
    // only the RDB final-conv instantiations carry it (it costs registers)
    static constexpr int FOLD = FOLD_;
    // 1: double-buffered fragment registers across (k-step, dx) steps; 2: the next step's reads
    // spread over the current step's MFMAs (front-loading them instead: 0.43-0.92x, register
    // pressure)
    static constexpr int PIPE = PIPE_;
    static constexpr int EPQ = EPQ_;   // epilogue operand units (8 VGPRs each) loaded per pass
    // refill placement: 0 = the next chunk's LDS-DMA issued right after the current chunk's
    // step-0 fragment reads (PIPE 2; otherwise as 1), 1 = issued before them (round-1 order),
    // > 1 = issued in SPL parts, one before each of the first SPL steps
    static constexpr int SPL = SPL_;
    // tap window: 0 = all 3x3 taps; 1 = taps {0,1}^2; 2 = taps {1,2}^2 (the 2x2 convs that a
    // stride-2 3x3 conv and its transpose become on the 2x2 phase decomposition, isr_conv_desc.taps)
    static constexpr int TWN = TWN_;
    static constexpr int TLO = TWN == 2 ? 1 : 0;
    static constexpr int TN = TWN ? 2 : 3;
    static constexpr int NA = R + TN - 1;  // input rows one wave reads per step
    static constexpr int CIN = CIN_; // 0 = runtime cin; else compile-time (own symbol)
    // Ablation bits, tuning builds only (outputs wrong): 1 = no MFMA (operands
    // kept live), 2 = stage only chunk 0 (no refill), 4 = no epilogue stores, 8 = the weights of
    // chunk 0 only (later chunks refill their halo but not their weights: the time a block would
    // take with its weights resident in LDS, round 6 probe for the Scaler / VGG short-K convs).
    static constexpr int ABL = ABL_;
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
    // NSW > 0: separate rings — halo planes NST deep (NST-1 chunks in flight), weights NSW deep
    // (one chunk ahead): the growth convs keep two halo chunks in flight at two blocks per CU
    static constexpr int NSW = NSW_;
    static constexpr int IPWH = (HALO_INSTR + WM - 1) / WM; // halo glds per wave per chunk
    static constexpr int IPWW = (W_INSTR + WM - 1) / WM;    // weight glds per wave (the last
                                                            // round repeats pieces: same bytes)
    static constexpr int HSTAGE = HALO_INSTR * 1024;
    static constexpr int WSTAGE = W_INSTR * 1024;
    static constexpr int RING = NSW ? NST * HSTAGE + NSW * WSTAGE : NST * STAGE;
    static constexpr int NT = 64 * WM;
    static constexpr int EPS = CT + 4;                 // floats per pixel in the epilogue image
    static constexpr int EP_BYTES = WM * 32 * EPS * 4; // one output row per wave at a time
    static constexpr int LDS = (RING > EP_BYTES) ? RING : EP_BYTES;
    static_assert(!NSW || (HALO_INSTR % WM == 0 && NST >= 3 && NSW == 2), "split rings");
    static constexpr int BPC = 163840 / LDS; // blocks per CU by LDS
    static constexpr int OCC = BPC * WM / 4 >= 2 ? 2 : 1; // waves per SIMD to budget registers for
    static_assert(LDS <= 163840, "LDS budget");
    static_assert(KC == 16 || KC == 32, "chunk width");
};

template <int V> struct IC { static constexpr int value = V; };

// 1: s_setprio 1 around each chunk's MFMA steps (as the trunk kernel): measured slower on the
// SRGAN step, 54.43 / 54.53 vs 53.95 / 54.21 ms same box (profiles/r03_train_conv_prio_ab.jsonl)
#ifndef ISR_CONV_PRIO
#define ISR_CONV_PRIO 0
#endif

// A operand of the residual fold: (1/s1) I on couts [16 h16, 16 h16 + 16) of a 32-cout
// fragment (lane l supplies A[l & 31][8 (l >> 5) .. + 8]); trunk.hip builds the same.
template <bool H>
__device__ __forceinline__ uint32_t fold_idv(float s1) {  // storage-type bits of 1/s1, in an SGPR
    return __builtin_amdgcn_readfirstlane((uint32_t)bits16<H>(1.f / s1));
}
__device__ __forceinline__ bf16x8 fold_a(uint32_t idv, int h16) {
    int lane = threadIdx.x & 63;
    // opaque to the optimiser: built next to its one use instead of hoisted out of the chunk
    // loop (two hoisted operands = 8 VGPRs the 256-VGPR final-conv kernel does not have)
    asm volatile("" : "+v"(lane));
    const int j = (lane & 31) - 16 * h16 - 8 * (lane >> 5);
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    u32x4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = j == 2 * k ? idv : (j == 2 * k + 1 ? idv << 16 : 0u);
    return __builtin_bit_cast(bf16x8, r);
}

// The fold applies when r1 is exactly the conv's own input channels [0, cout) (one cout tile),
// the activation is the identity and 1/s1 is exact in bf16 (add_rate 0.2 → 5).
template <class C, bool XS2, class Desc>
__device__ __forceinline__ bool fold_ok(const Desc& d) {
    if constexpr (!C::FOLD || C::NF != 2 || C::KS != 1 || C::TN != 3 || C::PIPE != 2 || XS2) {
        return false;
    } else {
        if (!d.r1.data || d.r1.data != d.x.data || d.r1.coff != d.x.coff || d.r1_cn != 0) return false;
        if (d.cout != C::CT || d.slope != 1.f || d.y2.data || d.m.data || d.shuffle != 1) return false;
        const float inv = 1.f / d.s1;
        if constexpr (C::H) return (float)(_Float16)inv == inv;
        else return (float)(__bf16)inv == inv;
    }
}

// Epilogue.  Accumulators are D[cout][pixel]: lane l owns pixel l31 of the row
// and couts (g&3) + 8*(g>>2) + 4*hh of each 32-cout fragment; the bias is
// already in them (accumulator init).
//  * plain stores (MODE 0..7): two v_permlane32_swap rounds per fragment give
//    every lane 8 contiguous couts twice, so each store is 16 bytes and one
//    store instruction covers 32 pixels x 32 contiguous bytes; no LDS, no
//    barrier.  All residual loads of a row are issued before its stores (the
//    output may alias a residual: the in-place RRDB update).
//  * PixelShuffle(2) (MODE 8): transpose through LDS one row at a time, so a
//    lane stores 8 channels of one shuffled output pixel.
// MODE bits (compile-time: no per-element branches): 1 = r1, 2 = r2, 4 = y2, 8 = shuffle,
// 16 = LeakyReLU' mask (backward).  r1_cn / m_c0 are multiples of 32, so their
// channel tests are uniform per 32-cout fragment (scalar branches).
template <class C, int MODE, int HX, class Desc>
__device__ __forceinline__ void epilogue(const Desc& d, f32x16 (&acc)[C::R][C::NF], int img, int ct,
                                         int x0, int y0, int wave, int lane) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = C::R, NF = C::NF, CT = C::CT, EPS = C::EPS;
    const int l31 = lane & 31, hh = lane >> 5;
    const float slope = d.slope;
    if constexpr (MODE & 8) {
        constexpr int ITEMS = CT / 16; // items (8 channels of one shuffled pixel) per lane per row
        constexpr int CG = CT / 32;
        float* ep = reinterpret_cast<float*>(smem) + wave * (32 * EPS);
        const int cg = lane % CG;
        const int sj = (lane / CG) & 1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            // registers 4j..4j+3 are 4 consecutive couts (the 4 sub-pixels of one shuffled
            // channel): one 16-byte write each (lane units 17·l31 + 2j + hh: conflict-free)
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x4 q = {acc[r][f][4 * j], acc[r][f][4 * j + 1], acc[r][f][4 * j + 2], acc[r][f][4 * j + 3]};
                    *reinterpret_cast<f32x4*>(ep + l31 * EPS + f * 32 + 8 * j + 4 * hh) = q;
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const int yy = y0 + wave * R + r;
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                // item → sub-row si (compile-time), output column xo, channel group cg
                const int si = it / CG;
                const int xo = (lane / CG + 64 * it / CG) & 63;
                const int xc = xo >> 1;
                float v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    v[k] = ep[xc * EPS + 4 * (cg * 8 + k) + 2 * si + sj];
                    v[k] = v[k] >= 0.f ? v[k] : v[k] * slope;
                }
                if constexpr (MODE & 16) {  // LeakyReLU' of the (shuffled-grid) mask source, all channels
                    const bf16x8 mq =
                        load16_hx<HX>(d.m, d.n, view_at(d.m, img, 2 * yy + si, 2 * x0 + xo, ct * (CT / 4) + cg * 8));
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (!(elt<C::H>(mq, k) > 0.f)) v[k] *= d.mslope;
                }
                if (!(yy < d.h && x0 + xc < d.w)) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = 0.f;
                }
                store8_bf16_hx<HX, C::H>(d.y, d.n, view_at(d.y, img, 2 * yy + si, 2 * x0 + xo, ct * (CT / 4) + cg * 8), v);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        const int xx = x0 + l31;
        // Residual / mask operands are loaded U (row, fragment) units at a time,
        // all loads of a pass before any of its stores, so the epilogue waits
        // for memory R*NF/U times instead of once per unit.  U is sized so the
        // operand registers stay at <= 32 VGPRs beside the 128 accumulators.
        // Loads of a unit precede its stores (in-place RRDB update: y may alias r1/r2).
        constexpr int P = ((MODE & 1) ? 1 : 0) + ((MODE & 2) ? 1 : 0) + ((MODE & 16) ? 1 : 0);
        constexpr int NU = R * NF;
        constexpr int U0 = P == 0 ? 1 : (C::EPQ / P > 0 ? C::EPQ / P : 1);
        constexpr int U = U0 > NU ? NU : U0;
        static_assert(NU % U == 0, "units per pass");
        bf16x8 q1[U][2], q2[U][2], qm[U][2];
        auto load_unit = [&](int uu, int buf) {
            const int r = uu / NF, f = uu % NF;
            const int yy = y0 + wave * R + r;
            const int cf = ct * CT + f * 32;
            const bool use_r1 = (MODE & 1) && (d.r1_cn == 0 || cf < d.r1_cn);
            const bool use_m = (MODE & 16) && cf >= d.m_c0;
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                const int co = cf + 16 * blk + 8 * hh;
                if constexpr (MODE & 1) {
                    if (use_r1) q1[buf][blk] = load16_hx<HX>(d.r1, d.n, view_at(d.r1, img, yy, xx, co));
                }
                if constexpr (MODE & 2) q2[buf][blk] = load16_hx<HX>(d.r2, d.n, view_at(d.r2, img, yy, xx, co));
                if constexpr (MODE & 16) {
                    if (use_m) qm[buf][blk] = load16_hx<HX>(d.m, d.n, view_at(d.m, img, yy, xx, co));
                }
            }
        };
        const bool scale2 = d.s2 != 1.f;  // s2 also scales when there is no r2 (backward)
#pragma unroll
        for (int uu = 0; uu < NU; ++uu) {
            const int r = uu / NF, f = uu % NF, cb = uu % U;
            const int yy = y0 + wave * R + r;
            const bool valid = yy < d.h && xx < d.w;
            if constexpr (P > 0) {
                if (cb == 0) {
#pragma unroll
                    for (int i = 0; i < U; ++i) load_unit(uu + i, i);
                }
            }
            const int cf = ct * CT + f * 32;
            const bool use_r1 = (MODE & 1) && (d.r1_cn == 0 || cf < d.r1_cn);
            const bool use_m = (MODE & 16) && cf >= d.m_c0;
            float v[16];
#pragma unroll
            for (int g = 0; g < 16; ++g) v[g] = acc[r][f][g];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                swap_halves(v[k], v[4 + k]);
                swap_halves(v[8 + k], v[12 + k]);
            }
            // v[8*blk + e] = cout f*32 + 16*blk + 8*hh + e
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                float* u = v + 8 * blk;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    u[e] = u[e] >= 0.f ? u[e] : u[e] * slope;
                    if constexpr (MODE & 32) u[e] = u[e] * d.s1;
                    if constexpr (MODE & 1) u[e] = u[e] * d.s1 + (use_r1 ? elt<C::H>(q1[cb][blk], e) : 0.f);
                    if constexpr (MODE & 2) {
                        u[e] = u[e] * d.s2 + elt<C::H>(q2[cb][blk], e);
                    } else {
                        if (scale2) u[e] *= d.s2;
                    }
                    if constexpr (MODE & 16) {
                        if (use_m && !(elt<C::H>(qm[cb][blk], e) > 0.f)) u[e] *= d.mslope;
                    }
                    if (!valid) u[e] = 0.f;
                }
                const int co = cf + 16 * blk + 8 * hh;
                store8_bf16_hx<HX, C::H>(d.y, d.n, view_at(d.y, img, yy, xx, co), u);
                if constexpr (MODE & 4) store8_bf16_hx<HX, C::H>(d.y2, d.n, view_at(d.y2, img, yy, xx, co), u);
            }
        }
    }
}

// Packed weights (isr_pack_conv3x3): [c16 = cin/16][tap 9][cout][hpos 2][8 bf16],
// element = W[n][c16*16 + h*8 + e][tap], h = hpos ^ ((n >> 3) & 1).
// XS2: the input is read as PixelShuffle(2)ᵀ (isr_conv_desc.x_sub2) — a template flag so the
// common path carries no per-chunk address division.
// One output tile (logical tile index t: cout tile innermost, then x, y, image) of the conv
// described by `d`, computed by the whole workgroup.  HX = 1 (the persistent chain kernel,
// conv_chain.hip): activations written by other workgroups of the same launch are read with
// sc1 loads (L1 bypass) and the outputs stored write-through (sc1), Guideline 16's hand-off.
struct NoPre {
    __device__ void operator()() const {}
};

// pre(): run after the tile's scalar setup (descriptor loads, addresses, bias loads) is issued
// and before its first LDS-DMA (the chain's dependency wait: the setup's memory latency then
// overlaps the wait); with early0 the first NST-1 chunks are staged before pre() (the chain,
// when those input channels were not written by the previous layer).
template <class C, bool XS2, int HX, class Desc, class Pre = NoPre>
__device__ __forceinline__ void conv_tile(const Desc& d, int t, int srow = -1, const Pre& pre = Pre{},
                                          bool early0 = false) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = C::R, NF = C::NF, WM = C::WM;

    const int nct = d.cout / C::CT;
    const int nbx = d.wa / C::TW, nby = d.ha / C::TH;
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
    // RDB residual fold (trunk.hip): when r1 is the conv's own input channels [0, cout) and the
    // activation is the identity, x/s1 is added by extra MFMAs on the staged centre pixels
    // (A = (1/s1) I, exact in bf16) and the epilogue computes acc * s1 — no r1 re-read.  The
    // same MFMA order as trunk.hip's kernel, so every path stays bit-identical.
    const bool fold = fold_ok<C, XS2>(d);
    const uint32_t fidv = C::FOLD ? fold_idv<C::H>(d.s1) : 0u;
    conv_stamp(0, srow);

    // ---- per-lane glds source offsets (chunk-invariant) -------------------
    // x_sub2 (backward of PixelShuffle): halo pixel (row, col) of sub-position s
    // lives at x pixel (2row + (s>>1), 2col + (s&1)) — pixel stride 2 plus a
    // per-chunk offset.
    const int ps = XS2 ? 2 : 1;
    const char* xbase = view_at(d.x, img, ps * (y0 - 1), ps * (x0 - 1), 0);
    const size_t pstride = plane_bytes(d.x);
    const char* wbase = (const char*)d.wpack;
    const int xrow_bytes = d.x.wp * 32;
    auto xchunk = [&](int chunk) -> size_t {
        if constexpr (!XS2) return (size_t)chunk * C::KS * pstride;
        const int cs4 = d.cin >> 2;
        const int c0 = chunk * C::KC;
        const int sp = c0 / cs4, cb = (c0 - sp * cs4) >> 4;
        return (size_t)cb * pstride + (size_t)(sp >> 1) * xrow_bytes + (sp & 1) * 32;
    };
    const size_t wchunk_bytes = (size_t)C::KS * 9 * d.cout * 32;
    // recomputed per stage instead of held in IPW registers (the wide kernel sits at the
    // 256-VGPR limit of two waves per SIMD)
    auto off_of = [&](int k) -> uint32_t {
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
                o = (uint32_t)(kp * pstride + ps * (row * xrow_bytes + col * 32) + c * 16);
            }
        } else if (j < C::INSTR) {
            const int u = (j - C::HALO_INSTR) * 64 + lane;
            const int seg = u / (C::CT * 2); // (ks, tap)
            const int rem = u - seg * (C::CT * 2);
            o = (uint32_t)((seg * d.cout + ct * C::CT) * 32 + rem * 16);
        }
        return o;
    };

    // split rings (NSW): halo pieces j = wave + WM*k (k < IPWH) and weight pieces jj = (wave + WM*k) %
    // W_INSTR (k < IPWW; the wrap repeats a piece: the same bytes to the same LDS address)
    auto stage_h = [&](int chunk, int buf) {
        char* dst = smem + buf * C::HSTAGE;
        const char* xs = xbase + xchunk(chunk);
#pragma unroll
        for (int k = 0; k < C::IPWH; ++k) {
            const int j = wave + WM * k;
            const uint32_t o = off_of(k);
            if constexpr (HX) glds16_sc1(xs + o, dst + j * 1024);
            else glds16(xs + o, dst + j * 1024);
        }
    };
    auto stage_w = [&](int chunk, int buf) {
        char* dst = smem + C::NST * C::HSTAGE + buf * C::WSTAGE;
        const char* ws = wbase + (size_t)chunk * wchunk_bytes;
#pragma unroll
        for (int k = 0; k < C::IPWW; ++k) {
            const int jj = (wave + WM * k) % C::W_INSTR;
            const int u = jj * 64 + lane;
            const int seg = u / (C::CT * 2);
            const int rem = u - seg * (C::CT * 2);
            glds16(ws + (uint32_t)((seg * d.cout + ct * C::CT) * 32 + rem * 16), dst + jj * 1024);
        }
    };
    auto stage = [&](int chunk, int buf, int k0 = 0, int k1 = C::IPW) {
        char* dst = smem + buf * C::STAGE;
        const char* xs = xbase + xchunk(chunk);
        const char* ws = wbase + (size_t)chunk * wchunk_bytes;
#pragma unroll
        for (int k = k0; k < k1; ++k) {
            const int j = wave + WM * k;
            const uint32_t o = off_of(k);
            if (j < C::HALO_INSTR) {
                if constexpr (HX) glds16_sc1(xs + o, dst + j * 1024);
                else glds16(xs + o, dst + j * 1024);
            } else if (!(C::ABL & 8) || chunk == 0) {
                glds16(ws + o, dst + j * 1024);
            }
        }
    };

    // D[cout][pixel] accumulators (A = weights, B = pixels): register g of lane l
    // holds cout f*32 + (g&3) + 8*(g>>2) + 4*hh of pixel l31; the bias is the init.
    f32x16 acc[R][NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        f32x16 b0;
#pragma unroll
        for (int g = 0; g < 16; ++g)
            b0[g] = d.bias ? d.bias[ct * C::CT + f * 32 + (g & 3) + 8 * (g >> 2) + 4 * hh] : 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][f] = b0;
    }

    auto prologue = [&]() {
        if constexpr (C::NSW) {  // issue order h(0), w(0), h(1), ..., h(NST-2): see the chunk wait
            stage_h(0, 0);
            stage_w(0, 0);
#pragma unroll
            for (int s = 1; s < C::NST - 1; ++s)
                if (s < nchunks) stage_h(s, s);
        } else {
#pragma unroll
            for (int s = 0; s < C::NST - 1; ++s)
                if (s < nchunks) stage(s, s);
        }
    };
    if (early0) prologue();
    pre();
    if (!early0) prologue();
    conv_stamp(5, srow);

    const int qw = wave * R * C::HC + l31; // halo pixel of (row w*R, col l31)
    // one K-chunk; FC = the chunk index (0..3) when the residual fold adds its MFMAs to this chunk,
    // -1 otherwise (the fold's chunks are peeled so that its accumulator choice is compile-time:
    // a run-time choice made hipcc copy a 16-VGPR accumulator and spill the 192->64 kernel)
    auto do_chunk = [&](const int chunk, auto fc_tag) {
        constexpr int FC = decltype(fc_tag)::value;
        (void)FC;
            // chunk `chunk` landed for this wave: younger chunks in flight = min(NST-2, nchunks-1-chunk)
            if constexpr (C::NSW) {
                // issue order ... w(c-1) h(c+1) | w(c) h(c+2) ...: at chunk c only the halo pieces of
                // chunk c+1 (issued after w(c)) may still be in flight (NST == 3)
                static_assert(C::NSW == 0 || C::NST == 3, "split-ring wait assumes NST 3");
                if (chunk + 1 < nchunks) {
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::IPWH) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            } else if constexpr (C::NST >= 3) {
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
            if (chunk == 0) conv_stamp(1, srow);
            const bool refill = !(C::ABL & 2) && chunk + C::NST - 1 < nchunks;
            // split rings: w(chunk+1) then h(chunk+NST-1), each when it exists
            auto refill_split = [&]() {
                if (chunk + 1 < nchunks) stage_w(chunk + 1, (chunk + 1) % C::NSW);
                if (refill) stage_h(chunk + C::NST - 1, (chunk + C::NST - 1) % C::NST);
            };
            if constexpr (C::SPL == 1 || (C::SPL == 0 && C::PIPE != 2)) {
                if constexpr (C::NSW) refill_split();
                else if (refill) stage(chunk + C::NST - 1, (chunk + C::NST - 1) % C::NST);
            }

            const char* hs = C::NSW ? smem + (chunk % C::NST) * C::HSTAGE
                                    : smem + ((C::ABL & 2) ? 0 : (chunk % C::NST)) * C::STAGE;
            const char* ws = C::NSW ? smem + C::NST * C::HSTAGE + (chunk % (C::NSW ? C::NSW : 1)) * C::WSTAGE
                                    : hs + C::HALO_INSTR * 1024;
            // Software pipeline over the chunk's (k-step, dx) steps: the fragments of
            // step st+1 are read into the other register set while step st's MFMAs
            // run, so LDS latency is covered by MFMA work of the same wave.
            constexpr int NS = C::KS * C::TN;
            constexpr int TN = C::TN, TLO = C::TLO, NA = C::NA;
            bf16x8 fb[2][TN][NF], fa[2][NA];
            auto load_step = [&](int st, int set) {
                const int ks = st / TN, dx = TLO + st % TN;
                const char* hp = hs + ks * C::HIPL * 1024;
    #pragma unroll
                for (int dyi = 0; dyi < TN; ++dyi)
    #pragma unroll
                    for (int f = 0; f < NF; ++f) {
                        const int n = f * 32 + l31;
                        const int u = ((ks * 9 + (TLO + dyi) * 3 + dx) * C::CT + n) * 2 + (hh ^ ((n >> 3) & 1));
                        fb[set][dyi][f] = lds_read16(ws + u * 16);
                    }
    #pragma unroll
                for (int ia = 0; ia < NA; ++ia) {
                    const int q = qw + (TLO + ia) * C::HC + dx;
                    fa[set][ia] = lds_read16(hp + halo_unit2(q, hh) * 16);
                }
            };
            // one fragment of step st: idx < TN*NF → weights (dyi, f), else activation row ia
            auto read_one = [&](int st, int idx, int set) {
                const int ks = st / TN, dx = TLO + st % TN;
                if (idx < TN * NF) {
                    const int dyi = idx / NF, f = idx % NF;
                    const int n = f * 32 + l31;
                    const int u = ((ks * 9 + (TLO + dyi) * 3 + dx) * C::CT + n) * 2 + (hh ^ ((n >> 3) & 1));
                    fb[set][dyi][f] = lds_read16(ws + u * 16);
                } else {
                    const int ia = idx - TN * NF;
                    int qb = qw;
                    // fold kernels: the row's swizzled address is recomputed at each read (an opaque
                    // copy of qw) — hoisted, the peeled fold chunks kept ~18 of them live and spilled
                    if constexpr (C::FOLD) asm volatile("" : "+v"(qb));
                    const int q = qb + (TLO + ia) * C::HC + dx;
                    fa[set][ia] = lds_read16(hs + ks * C::HIPL * 1024 + halo_unit2(q, hh) * 16);
                }
            };
            if constexpr (C::PIPE) load_step(0, 0);
            if constexpr (C::PIPE == 2) {
                // the refill's LDS-DMA issue (10-16 instructions, scalar address math) runs while
                // step 0's fragment reads are in flight, instead of ahead of them
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (C::SPL == 0) {
                    if constexpr (C::NSW) refill_split();
                    else if (refill) stage(chunk + C::NST - 1, (chunk + C::NST - 1) % C::NST);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
    #if ISR_CONV_PRIO
            __builtin_amdgcn_s_setprio(1);  // A/B: the MFMA steps ahead of the co-resident block's issue
#endif
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                const int cur = C::PIPE ? (st & 1) : 0;
                if constexpr (C::SPL > 1) {
                    static_assert(C::SPL <= NS, "refill parts must fit the chunk's steps");
                    if (st < C::SPL && refill)
                        stage(chunk + C::NST - 1, (chunk + C::NST - 1) % C::NST, st * C::IPW / C::SPL,
                              (st + 1) * C::IPW / C::SPL);
                }
                if constexpr (C::PIPE == 2) {
                    // interleaved: this step's MFMAs with the next step's fragment reads (one
                    // read after each MFMA), so at most one step's reads are in flight (<= 15,
                    // the lgkmcnt range: beyond it hipcc can only wait lgkmcnt(0))
                    constexpr int NRD = TN * NF + NA;  // reads per step
                    constexpr int NM = R * TN * NF;    // MFMAs per step
                    int m = 0;

    #pragma unroll
                    for (int ia = 0; ia < NA; ++ia) {
    #pragma unroll
                        for (int dyi = 0; dyi < TN; ++dyi) {
                            const int r = ia - dyi;
                            if (r >= 0 && r < R) {
    #pragma unroll
                                for (int f = 0; f < NF; ++f) {
                                    acc[r][f] = mfma32t<C::H>(fb[cur][dyi][f], fa[cur][ia], acc[r][f]);
                                    if (st + 1 < NS)
                                        for (int k = m * NRD / NM; k < (m + 1) * NRD / NM; ++k) read_one(st + 1, k, cur ^ 1);
                                    __builtin_amdgcn_sched_barrier(0);  // pin the (MFMA, reads) order
                                    ++m;
                                }
                            }
                        }
                        if constexpr (FC >= 0 && C::FOLD && C::NF == 2 && C::KS == 1 && C::TN == 3) {
                            // residual fold: + x/s1 on the centre pixels of output row ia - 1 (dx = 1,
                            // dy = 1), right after input row ia's MFMAs (trunk.hip's order); the chunk
                            // (0..3) is a compile-time constant here, so the target accumulator is too
                            if (st == 1 && ia >= 1 && ia <= R) {
                                const bf16x8 a = fold_a(fidv, FC & 1);
                                acc[ia - 1][FC >> 1] = mfma32t<C::H>(a, fa[cur][ia], acc[ia - 1][FC >> 1]);
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        }
                    }
                    continue;
                } else if constexpr (C::PIPE) {
                    if (st + 1 < NS) load_step(st + 1, cur ^ 1);
                    // keep the prefetch ahead of this step's MFMAs (hipcc otherwise sinks
                    // each ds_read next to its first use and waits lgkmcnt(0) there)
                    __builtin_amdgcn_sched_barrier(0);
                } else {
                    load_step(st, 0);
                }
                // input row TLO+ia feeds output row r through kernel row dy = TLO+dyi: r = ia - dyi
    #pragma unroll
                for (int ia = 0; ia < NA; ++ia) {
    #pragma unroll
                    for (int dyi = 0; dyi < TN; ++dyi) {
                        const int r = ia - dyi;
                        if (r >= 0 && r < R) {
    #pragma unroll
                            for (int f = 0; f < NF; ++f) {
                                if constexpr (C::ABL & 1) {
                                    asm volatile("" ::"v"(fa[cur][ia]), "v"(fb[cur][dyi][f]));
                                } else {
                                    acc[r][f] = mfma32t<C::H>(fb[cur][dyi][f], fa[cur][ia], acc[r][f]);
                                }
                            }
                        }
                    }
                }
            }
#if ISR_CONV_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
    };
    int chunk0 = 0;
    if constexpr (C::FOLD && C::NF == 2 && C::KS == 1 && C::TN == 3) {
        if (fold && nchunks >= 4) {
            do_chunk(0, IC<0>{});
            do_chunk(1, IC<1>{});
            do_chunk(2, IC<2>{});
            do_chunk(3, IC<3>{});
            chunk0 = 4;
        }
    }
    // not unrolled: with a compile-time cin (the 192->64 kernels) hipcc unrolled all 12 chunk bodies
    // and spilled 476 B/lane (108 vs 72 us per call)
#pragma nounroll
    for (int chunk = chunk0; chunk < nchunks; ++chunk) do_chunk(chunk, IC<-1>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier(); // all waves done reading the ring before it becomes the epilogue image
    conv_stamp(2, srow);

    if constexpr (C::ABL & 4) {
        if (d.n < 0) { // never true: keeps the accumulators (and so the MFMAs) live
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int f = 0; f < NF; ++f)
#pragma unroll
                    for (int g = 0; g < 16; ++g) s += acc[r][f][g];
            ((float*)d.y.data)[threadIdx.x] = s;
        }
        return;
    }
    // ---- epilogue (mode picked once, wave-uniform, so no per-element branches)
    const int mode = d.shuffle == 2 ? (d.m.data ? 24 : 8)
                     : fold ? (32 | (d.r2.data ? 2 : 0))
                            : ((d.r1.data ? 1 : 0) | (d.r2.data ? 2 : 0) | (d.y2.data ? 4 : 0) | (d.m.data ? 16 : 0));
    if constexpr (HX) {  // chain layers: growth (plain store) or the RDB final conv (folded r1 [+ r2])
        if (mode == 0) epilogue<C, 0, HX>(d, acc, img, ct, x0, y0, wave, lane);
        else if (mode == 32) epilogue<C, 32, HX>(d, acc, img, ct, x0, y0, wave, lane);
        else if (mode == 34) epilogue<C, 34, HX>(d, acc, img, ct, x0, y0, wave, lane);
        else if (mode == 1) epilogue<C, 1, HX>(d, acc, img, ct, x0, y0, wave, lane);
        else epilogue<C, 3, HX>(d, acc, img, ct, x0, y0, wave, lane);
    } else switch (mode) {
        case 32: epilogue<C, 32, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 34: epilogue<C, 34, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 0: epilogue<C, 0, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 1: epilogue<C, 1, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 2: epilogue<C, 2, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 3: epilogue<C, 3, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 4: epilogue<C, 4, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 5: epilogue<C, 5, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 6: epilogue<C, 6, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 7: epilogue<C, 7, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 8: epilogue<C, 8, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 24: epilogue<C, 24, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 16: epilogue<C, 16, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 17: epilogue<C, 17, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 18: epilogue<C, 18, HX>(d, acc, img, ct, x0, y0, wave, lane); break;
        default: epilogue<C, 19, HX>(d, acc, img, ct, x0, y0, wave, lane); break;  // 19; y2 + mask is rejected by isr_conv3x3_fwd
    }
#ifdef ISR_TUNING
    if (srow == -1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        conv_stamp(3, srow);
    }
#endif
}

template <class C, bool XS2>
__global__ __launch_bounds__(C::NT, C::OCC) void conv3x3_fwd_kernel(isr_conv_desc d) {
    conv_tile<C, XS2, 0>(d, xcd_remap(blockIdx.x, gridDim.x));
}

template <class C, bool XS2>
static int launch3x3_k(const isr_conv_desc* d, hipStream_t s) {
    auto kern = conv3x3_fwd_kernel<C, XS2>;
    lds_limit((const void*)kern, C::LDS);
    const int blocks = (d->wa / C::TW) * (d->ha / C::TH) * d->n * (d->cout / C::CT);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(C::NT), C::LDS, s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// FULL: the production tiles also carry the PixelShuffleᵀ-input form; the A/B variants
// take the plain form only (x_sub2 → unsupported).
template <class C, bool FULL = false>
static int launch3x3(const isr_conv_desc* d, hipStream_t s) {
    if (d->cout % C::CT || d->cin % C::KC || d->ha % C::TH) return -2;
    if (C::CIN && d->cin != C::CIN) return -2;
    if constexpr (FULL) {
        if (d->x_sub2) return launch3x3_k<C, true>(d, s);
    } else {
        if (d->x_sub2) return -2;
    }
    return launch3x3_k<C, false>(d, s);
}

// Variant table: variant 0 is the production choice per shape; the others are
// kept for on-device A/B tuning (isr_conv3x3_fwd_variant, tools/tune_conv.py).
// (tools/tune_conv.py on MI355X, N=16 128²: the 16x32-tile, 2-blocks/CU configs are
// fastest on every shape of the generator; the 32x32 8-wave tiles win only at long K)
// cout == 32 (RDB growth convs)
// V_G0 / V_F0: the next step's fragment reads interleaved one per MFMA (PIPE 2): 2-7 % over the
// batched prefetch, whose 18-24 reads in flight exceed lgkmcnt's range (so hipcc waited lgkmcnt(0))
using V_G0 = C3<4, 4, 1, 16, 2, 0, 0, 2>; // 16x32, 4 waves, KC16 double buffer, 58 KB → 2 blocks / CU
using V_G1 = C3<4, 8, 1, 16, 3>; // 32x32 px tile, 8 waves, 3-deep KC16 ring
using V_G2 = C3<2, 4, 1, 32, 2>; // 8x32, KC32, 2 blocks / CU
using V_G3 = C3<2, 4, 1, 16, 2, 0, 0, 2>; // 8x32 tile, double buffer, interleaved
// cout % 64 == 0
using V_W0 = C3<4, 4, 2, 16, 2, 0, 0, 2>; // 16x32, 4 waves, KC16 double buffer, 76 KB → 2 blocks / CU, PIPE 2
using V_W1 = C3<4, 8, 2, 16, 2>; // 32x32 px tile, 8 waves, KC16 double buffer
using V_W2 = C3<2, 4, 2, 32, 2>; // 8x32, KC32
using V_W3 = C3<2, 4, 2, 16, 2, 0, 0, 2>; // 8x32 tile, interleaved
using V_F0 = C3<4, 4, 2, 16, 2, 192, 0, 2>; // RDB final conv 192→64: V_W0 with compile-time cin, PIPE 2
using V_F0F = C3<4, 4, 2, 16, 2, 192, 0, 2, 4, 0, 0, 0, 1>; // V_F0 with the residual fold (r1 == x)
// fp16 storage (isr_conv_desc.f16: the inference path) — the same four production tiles
using V_G0H = C3<4, 4, 1, 16, 2, 0, 0, 2, 4, 0, 0, 0, 0, 1>;
using V_W0H = C3<4, 4, 2, 16, 2, 0, 0, 2, 4, 0, 0, 0, 0, 1>;
using V_F0H = C3<4, 4, 2, 16, 2, 192, 0, 2, 4, 0, 0, 0, 0, 1>;
using V_F0FH = C3<4, 4, 2, 16, 2, 192, 0, 2, 4, 0, 0, 0, 1, 1>;

// Host mirror of fold_ok: r1 is the conv's own input channels [0, cout), identity activation,
// 1/s1 exact in bf16 (its low 16 fp32 bits zero).
static bool fold_host(const isr_conv_desc* d) {
    if (!d->r1.data || d->r1.data != d->x.data || d->r1.coff != d->x.coff || d->r1_cn != 0) return false;
    if (d->cout != 64 || d->slope != 1.f || d->y2.data || d->m.data || d->shuffle != 1 || d->x_sub2 || d->taps)
        return false;
    const float inv = 1.f / d->s1;
    uint32_t bits;
    memcpy(&bits, &inv, 4);
    if (d->f16) {  // exact in fp16: 10 mantissa bits, a normal fp16 exponent
        const int ex = (int)((bits >> 23) & 0xff) - 127;
        return (bits & 0x1fffu) == 0 && ex >= -14 && ex <= 15;
    }
    return (bits & 0xffffu) == 0;
}

int conv3x3_fwd_variant(const isr_conv_desc* d, int variant, hipStream_t s) {
    if (d->f16) {  // fp16 storage: the production tiles only (the inference forward)
        if (variant != 0 || d->x_sub2 || d->taps || d->m.data) return -2;
        if (d->cout % 64) return launch3x3<V_G0H>(d, s);
        return d->cin == 192 ? (fold_host(d) ? launch3x3<V_F0FH>(d, s) : launch3x3<V_F0H>(d, s)) : launch3x3<V_W0H>(d, s);
    }
    if (d->cout % 64) {  // 32-cout tiles: growth convs (cout 32) and dgrad of them (96, 160)
        switch (variant) {
            case 0: return launch3x3<V_G0, true>(d, s);
#ifdef ISR_TUNING
            // A/B tile configurations (none faster than V_G0 on the generator's shapes)
            case 1: return launch3x3<V_G1>(d, s);
            case 2: return launch3x3<V_G2>(d, s);
            case 3: return launch3x3<V_G3>(d, s);
            case 8: return launch3x3<C3<4, 4, 1, 16, 2, 0, 0, 2, 4, 1>>(d, s);  // V_G0, refill before step-0 reads (r1)
            case 9: return launch3x3<C3<4, 8, 1, 16, 2, 0, 0, 2>>(d, s);  // 32x32 tile, 8 waves, PIPE 2 (92 KB, 1 block/CU)
            // ablations of V_G0 (timing only, outputs wrong): tuning builds only
            case 4: return launch3x3<C3<4, 4, 1, 16, 2, 0, 1>>(d, s);
            case 5: return launch3x3<C3<4, 4, 1, 16, 2, 0, 2>>(d, s);
            case 6: return launch3x3<C3<4, 4, 1, 16, 2, 0, 4>>(d, s);
            case 7: return launch3x3<C3<4, 4, 1, 16, 2, 0, 3>>(d, s);
#endif
        }
        return -2;
    }
    switch (variant) {
        case 0: return d->cin == 192 ? (fold_host(d) ? launch3x3<V_F0F>(d, s) : launch3x3<V_F0, true>(d, s))
                                     : launch3x3<V_W0, true>(d, s);
#ifdef ISR_TUNING
        case 1: return launch3x3<V_W1>(d, s);
        case 2: return launch3x3<V_W2>(d, s);
        case 3: return launch3x3<V_W3>(d, s);
        case 8: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 0, 2, 4, 1>>(d, s)  // refill before reads (r1)
                                     : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 2, 4, 1>>(d, s);
        case 9: return d->cin == 192 ? launch3x3<C3<4, 8, 2, 16, 2, 192, 0, 2>>(d, s)  // 32x32, 8 waves, PIPE 2 (111 KB)
                                     : launch3x3<C3<4, 8, 2, 16, 2, 0, 0, 2>>(d, s);
        // timing probes (outputs wrong): V_W0 / variant 9 without the weight refills (ABL 8)
        case 10: return launch3x3<C3<4, 4, 2, 16, 2, 0, 8, 2>>(d, s);
        case 11: return launch3x3<C3<4, 8, 2, 16, 2, 0, 8, 2>>(d, s);
        // ablations of V_W0 (timing only, outputs wrong): tuning builds only
        case 4: return launch3x3<C3<4, 4, 2, 16, 2, 0, 1>>(d, s);
        case 5: return launch3x3<C3<4, 4, 2, 16, 2, 0, 2>>(d, s);
        case 6: return launch3x3<C3<4, 4, 2, 16, 2, 0, 4>>(d, s);
        case 7: return launch3x3<C3<4, 4, 2, 16, 2, 0, 3>>(d, s);
#endif
    }
    return -2;
}

// ============ persistent chain: a run of RDB convs in ONE launch ============
// The RRDB trunk (utils/models.py:298-317, 245-271: per RDB four growth convs and the
// final 192→64 conv) as one persistent launch instead of one launch per conv.  Every
// layer shares the 16x32-pixel tile grid; workgroup b owns tiles b, b+G, ... for every
// layer (all G workgroups resident: G <= 2 per CU, the kernel's occupancy).  Tile t of
// layer L may start once tiles N(t) (itself and its 8 neighbours — the 3x3 halo) of layer
// L-1 are done: their progress words reach L.  That single stencil dependency also covers
// every older read/write hazard (a tile's layer-L-m ancestors within radius m are done).
// Hand-off (cdna_hip_programming.md Guideline 16, R1): outputs are stored write-through
// (sc1) and drained (s_waitcnt vmcnt(0) by every wave, barrier) before one lane publishes
// the progress word with a relaxed agent-scope atomic store; consumers poll relaxed
// (one lane per neighbour), then read the activations with sc1 loads (L1 bypass), and
// with `acquire` additionally run one agent-scope acquire per tile first.
// State (no per-call memset: a captured memset node was seen to leave garbage in the first
// words under HIP-graph replay): state[0] = generation, bumped by a one-thread kernel ahead of
// every chain launch; progress word of a tile = gen * 1024 + layers done (compared by serial-
// number arithmetic, so it never needs zeroing); a bounded spin that gives up writes the
// generation into state[1] (results invalid; the host checks state[1] == state[0]).
struct ChainArgs {
    const isr_conv_desc* layers;
    const int32_t* kinds;
    int nl, ntiles, nby, nbx;
    unsigned* state;
    int acquire;
};

#define CHAIN_STAMP_L0 75  // tuning stamps: the 15 layers of RRDB 5
// chain stamp rows start past every per-conv launch's blockIdx rows (those stamp at row
// blockIdx.x: up to 8192 for the x4 Scaler), so the later launches of a forward cannot
// overwrite them
#define CHAIN_STAMP_BASE 65536

#ifdef ISR_TUNING
// isr_tuning_chain_knobs: [0] start delay (s_memrealtime ticks, 100 MHz) of the workgroups whose
// bit [1] of blockIdx.x is set (a phase offset between independent image groups)
__device__ int g_chain_knobs[4];
#endif

__device__ __forceinline__ void chain_tuning_prologue(int ntiles) {
#ifdef ISR_TUNING
    unsigned long long* p = g_conv_stamps;
    if (p != nullptr && threadIdx.x == 0) {  // placement of every workgroup, after the 15 stamped layers
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); // HW_REG_XCC_ID
        p[((size_t)CHAIN_STAMP_BASE + 15 * ntiles + blockIdx.x) * 8 + 6] = hw;
        p[((size_t)CHAIN_STAMP_BASE + 15 * ntiles + blockIdx.x) * 8 + 7] = xcc;
    }
    const int dly = g_chain_knobs[0];
    if (dly > 0 && ((blockIdx.x >> g_chain_knobs[1]) & 1)) {
        unsigned long long t0, t;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
        do {
            __builtin_amdgcn_s_sleep(8);
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        } while (t - t0 < (unsigned long long)dly);
    }
#else
    (void)ntiles;
#endif
}

// The round-2 per-tile chain kernel (isr_conv_chain variant 1): superseded by trunk.hip, kept in the
// tuning library only (-DISR_TUNING).
#ifdef ISR_TUNING
__global__ void chain_bump_kernel(unsigned* state) {
    if (threadIdx.x == 0) state[threadIdx.x] = state[threadIdx.x] + 1u;  // vector store by lane 0
}

__device__ __forceinline__ void chain_wait(const ChainArgs& a, int t, unsigned need, unsigned gen) {
    unsigned* progress = a.state + 4;
    if (wave_id() == 0) {
        const int lane = threadIdx.x & 63;
        int nb = -1;
        if (lane < 9) {
            const int bx = t % a.nbx, by = (t / a.nbx) % a.nby, img = t / (a.nbx * a.nby);
            const int yy = by + lane / 3 - 1, xx = bx + lane % 3 - 1;
            if (yy >= 0 && yy < a.nby && xx >= 0 && xx < a.nbx) nb = (img * a.nby + yy) * a.nbx + xx;
        }
        for (unsigned spins = 0;; ++spins) {
            const bool ok =
                nb < 0 ||
                (int)(__hip_atomic_load(progress + nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - need) >= 0;
            if (__all(ok)) break;
            // a neighbour never arrived (not resident?): give up after ~0.3 s, flag it, and let
            // every later wait of the launch give up at once, so the grid always drains
            if ((spins & 255) == 255 &&
                __hip_atomic_load(a.state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen)
                break;
            if (spins > (1u << 18)) {
                if (lane == 0) {
                    __hip_atomic_store(a.state + 1, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(a.state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (a.acquire) {
            if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
}

typedef const __attribute__((address_space(4))) isr_conv_desc const_desc;  // constant memory:
// the host writes the layer table before the launch, so the compiler may re-load any field
// (s_load) instead of holding it in registers across the tile

// Static assignment: workgroup b owns tiles b, b+G, ... for every layer, so a tile's own
// previous-layer outputs were written by the same CU.  A queue dealing (layer, tile) items in
// layer order (no residency assumption) measured slower: 9.3 vs 6.8 ms per forward — it
// rebuilds a per-layer front and loses that locality.  All G workgroups must be resident
// (G <= 2 per CU); a wait that never completes gives up (bounded) instead of hanging.
// WM_: 0 = dependency wait before the tile; 1 = inside conv_tile after its scalar setup (the
// descriptor loads overlap the wait); 2 = as 1, and the first chunk is staged before the wait
// when the previous layer did not write those input channels (every layer but an RDB's first);
// 3 = as 1, and a tile's store drain + progress publish is deferred into the NEXT tile's pre(),
// after that tile's scalar setup (the write-through drain overlaps the setup's latency)
template <class CG, class CF, int WM_ = 0>
__global__ __launch_bounds__(CG::NT, 2) void conv_chain_kernel(ChainArgs a) {
    // bumped by chain_bump_kernel before this launch; an agent-scope load, so no CU reads a
    // stale copy of another XCD's write
    const unsigned gen = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    chain_tuning_prologue(a.ntiles);
    int pend_t = -1;  // WM_ 3: tile whose stores are not yet drained / published (uniform)
    unsigned pend_v = 0;
    auto publish_pending = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores are done
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(a.state + 4 + pend_t, pend_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend_t = -1;
    };
    for (int L = 0; L < a.nl; ++L) {
        const_desc& d = ((const_desc*)(uintptr_t)a.layers)[L];
        const int kind = a.kinds[L];
        for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
#ifdef ISR_TUNING
            const int srow =
                (L >= CHAIN_STAMP_L0 && L < CHAIN_STAMP_L0 + 15) ? CHAIN_STAMP_BASE + (L - CHAIN_STAMP_L0) * a.ntiles + t : -2;
#else
            const int srow = -2;
#endif
            conv_stamp(4, srow);  // wait start
            if constexpr (WM_ == 0) {
                if (L > 0) chain_wait(a, t, gen * 1024u + (unsigned)L, gen);
                if (kind == 0) conv_tile<CG, false, 1>(d, t, srow);
                else conv_tile<CF, false, 1>(d, t, srow);
            } else {
                bool early0 = false;
                if (WM_ == 2 && L > 0) {
                    // first-chunk input channels [x.coff, x.coff + 16) vs the previous layer's output
                    const_desc& dp = ((const_desc*)(uintptr_t)a.layers)[L - 1];
                    const int ech = 16 * (kind == 0 ? CG::NST - 1 : CF::NST - 1);  // channels staged early
                    early0 = !(dp.y.data == d.x.data && dp.y.coff < d.x.coff + ech && d.x.coff < dp.y.coff + dp.cout);
                }
                auto pre = [&]() {
                    if (WM_ == 3 && pend_t >= 0) publish_pending();
                    if (L > 0) chain_wait(a, t, gen * 1024u + (unsigned)L, gen);
                };
                if (kind == 0) conv_tile<CG, false, 1>(d, t, srow, pre, early0);
                else conv_tile<CF, false, 1>(d, t, srow, pre, early0);
                if constexpr (WM_ == 3) {
                    pend_t = t;
                    pend_v = gen * 1024u + (unsigned)(L + 1);
                    continue;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores are done
            conv_stamp(3, srow);
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_store(a.state + 4 + t, gen * 1024u + (unsigned)(L + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (pend_t >= 0) publish_pending();
}


#ifdef ISR_TUNING
static int g_chain_variant_host = 0;  // isr_tuning_chain_knobs k2: chain kernel variant (A/B only)
#endif

template <class CG, class CF, int WM_ = 0>
static int launch_chain(const isr_chain_desc* c, hipStream_t s) {
    static_assert(CG::TH == CF::TH && CG::TW == CF::TW, "one tile grid");
    static_assert(CG::NT == CF::NT, "one block size");
    if (c->ha % CG::TH || c->wa % CG::TW) return -2;
    ChainArgs a;
    a.layers = c->layers;
    a.kinds = c->kinds;
    a.nl = c->nl;
    a.nby = c->ha / CG::TH;
    a.nbx = c->wa / CG::TW;
    a.ntiles = c->n * a.nby * a.nbx;
    a.state = c->state;
    a.acquire = c->acquire;
    if (c->nl >= 1024) return -2;
    hipLaunchKernelGGL(chain_bump_kernel, dim3(1), dim3(64), 0, s, c->state);
    auto kern = conv_chain_kernel<CG, CF, WM_>;
    constexpr int lds = CG::LDS > CF::LDS ? CG::LDS : CF::LDS;
    lds_limit((const void*)kern, lds);
    int per_cu = 0;  // residency from the occupancy API (registers, LDS), capped at the 2 it is built for
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, CG::NT, lds) != hipSuccess) return -1;
    per_cu = per_cu < 2 ? per_cu : 2;
    if (per_cu < 1) return -1;
    const int slots = per_cu * cu_count();  // every workgroup resident
    const int grid = a.ntiles < slots ? a.ntiles : slots;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(CG::NT), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int conv_chain(const isr_chain_desc* c, hipStream_t s) {
#ifdef ISR_TUNING
    switch (g_chain_variant_host) {
        case 1:  // RDB final conv: every residual unit of a pass loaded at once (EPQ 8)
            return launch_chain<V_G0, C3<4, 4, 2, 16, 2, 192, 0, 2, 8>>(c, s);
        case 2:  // 32x32 tiles, 8 waves, 1 block / CU: growth 3-deep ring, final 2-deep
            return launch_chain<C3<4, 8, 1, 16, 3, 0, 0, 2>, C3<4, 8, 2, 16, 2, 192, 0, 2>>(c, s);
        case 3:  // 2 + EPQ 8
            return launch_chain<C3<4, 8, 1, 16, 3, 0, 0, 2>, C3<4, 8, 2, 16, 2, 192, 0, 2, 8>>(c, s);
        case 4:  // 32x32 tiles, both 2-deep
            return launch_chain<C3<4, 8, 1, 16, 2, 0, 0, 2>, C3<4, 8, 2, 16, 2, 192, 0, 2>>(c, s);
        case 9:  // deferred drain + publish (WM 3)
            return launch_chain<V_G0, V_F0, 3>(c, s);
        case 7:  // growth convs: split rings (halo 3 deep, weights 2 deep), wait after setup
            return launch_chain<C3<4, 4, 1, 16, 3, 0, 0, 2, 4, 0, 0, 2>, V_F0, 1>(c, s);
        case 8:  // 7 with the wait before the tile
            return launch_chain<C3<4, 4, 1, 16, 3, 0, 0, 2, 4, 0, 0, 2>, V_F0, 0>(c, s);
        case 5:  // the wait before the tile (the round-2 form; production waits after the setup)
            return launch_chain<V_G0, V_F0, 0>(c, s);
        case 6:  // 5 + first chunk staged before the wait where independent of the previous layer
            return launch_chain<V_G0, V_F0, 2>(c, s);
        default: break;
    }
#endif
    // production: the dependency wait runs after the tile's scalar setup (its descriptor loads —
    // three dependent scalar round trips, ~2.4 µs per tile — overlap the wait): -1.2 % per
    // forward against waiting first (tools/chain_probe.py, variant 0 vs 5)
    return launch_chain<V_G0, V_F0F, 1>(c, s);
}

#else
int conv_chain(const isr_chain_desc*, hipStream_t) { return -3; }
#endif  // ISR_TUNING (round-2 chain)

size_t conv_chain_state_words(int n, int ha, int wa) {
    const size_t tiles = (size_t)n * (ha / V_G0::TH) * (wa / V_G0::TW);
    return (tiles + 4 + 3) / 4 * 4;  // [0] fail word, [4..] progress; a multiple of 16 bytes
}

#ifdef ISR_TUNING
int conv_stamps_set(void* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_conv_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1; }
int chain_knobs_set(const int* k) {
    g_chain_variant_host = k[2];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_chain_knobs), k, 4 * sizeof(int)) == hipSuccess ? 0 : -1;
}
#else
int conv_stamps_set(void*) { return -2; }
int chain_knobs_set(const int*) { return -2; }
#endif

int conv3x3_fwd_dispatch(const isr_conv_desc* d, hipStream_t s) {
    if (d->f16) return conv3x3_fwd_variant(d, 0, s);
    if (d->taps == 1) return d->cout % 64 ? -2 : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 0, 4, 1, 1>, true>(d, s);
    if (d->taps == 2) return d->cout % 64 ? -2 : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 0, 4, 1, 2>, true>(d, s);
    return conv3x3_fwd_variant(d, 0, s);
}

// ---- weight packing: fp32 OIHW → bf16 [c16][tap][cout][hpos][8] -----------
// Forward: the packed conv has (cout, cin) = the layer's, element W[n][ci][tap].
// dgrad (transposed): the packed conv maps the layer's output gradient (cin' =
// layer cout) to its input gradient (cout' = layer cin): element
// scale * W[co(ci')][n][8 - tap] (180° rotation), where with sub2 the input
// channel ci' = s*(layer cout/4) + c stands for layer channel co = 4c + s
// (PixelShuffle order, see isr_conv_desc.x_sub2).
template <class OT = __bf16>
__device__ __forceinline__ void pack3x3_range(const float* __restrict__ w, OT* __restrict__ out, int pcout,
                                              int pcin, int transposed, int sub2, float scale, size_t first,
                                              size_t stride, int src_n0 = 0, int src_cin = 0) {
    // dgrad window: packed output channel n = layer input channel src_n0 + n of a layer with
    // src_cin input channels (row stride of w); 0 → the whole layer (src_cin = pcout)
    const int wrow = src_cin > 0 ? src_cin : pcout;
    const size_t total = (size_t)pcout * pcin * 9;
    for (size_t idx = first; idx < total; idx += stride) {
        size_t rem = idx;
        const int e = rem % 8; rem /= 8;
        const int hpos = rem % 2; rem /= 2;
        const int n = rem % pcout; rem /= pcout;
        const int tap = rem % 9; rem /= 9;
        const int c16 = (int)rem;
        const int h = hpos ^ ((n >> 3) & 1);
        const int ci = c16 * 16 + h * 8 + e;
        float v;
        if (!transposed) {
            v = w[((size_t)n * pcin + ci) * 9 + tap];
        } else {
            const int cs4 = pcin >> 2;
            const int co = sub2 ? (ci % cs4) * 4 + ci / cs4 : ci;  // layer output channel
            v = w[((size_t)co * wrow + src_n0 + n) * 9 + (8 - tap)];  // layer W[co][n0 + n][8 - tap]
        }
        out[idx] = (OT)(v * scale);
    }
}

template <class OT>
__global__ void pack3x3_kernel(const float* __restrict__ w, OT* __restrict__ out, int pcout, int pcin,
                               int transposed, int sub2, float scale) {
    pack3x3_range<OT>(w, out, pcout, pcin, transposed, sub2, scale, blockIdx.x * (size_t)blockDim.x + threadIdx.x,
                      (size_t)gridDim.x * blockDim.x);
}

// Many packs in one launch (the training plan repacks every conv each step):
// blockIdx.y = item, blockIdx.x strides over that item's elements.
__global__ void pack3x3_batch_kernel(const isr_pack_item* __restrict__ items) {
    const isr_pack_item it = items[blockIdx.y];
    const int pcout = it.dgrad ? it.cin : it.cout, pcin = it.dgrad ? it.cout : it.cin;
    pack3x3_range(it.w, (__bf16*)it.out, pcout, pcin, it.dgrad, it.sub2, it.dgrad ? it.scale : 1.f,
                  blockIdx.x * (size_t)blockDim.x + threadIdx.x, (size_t)gridDim.x * blockDim.x,
                  it.dgrad ? it.src_n0 : 0, it.dgrad ? it.src_cin : 0);
}

int conv3x3_pack_batch(const isr_pack_item* items, int n, hipStream_t s) {
    hipLaunchKernelGGL(pack3x3_batch_kernel, dim3(96, n), dim3(256), 0, s, items);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t conv3x3_packed_bytes(int cout, int cin) { return (size_t)cout * cin * 9 * 2; }

static int pack_launch(const float* w, void* out, int pcout, int pcin, int transposed, int sub2, float scale,
                       hipStream_t s) {
    const size_t total = conv3x3_packed_bytes(pcout, pcin) / 2;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(pack3x3_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, w, (__bf16*)out, pcout, pcin, transposed,
                       sub2, scale);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int conv3x3_pack(const float* w, void* out, int cout, int cin, hipStream_t s) {
    return pack_launch(w, out, cout, cin, 0, 0, 1.f, s);
}

// the forward pack in fp16 (isr_conv_desc.f16): same layout and size
int conv3x3_pack_f16(const float* w, void* out, int cout, int cin, hipStream_t s) {
    const size_t total = conv3x3_packed_bytes(cout, cin) / 2;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(pack3x3_kernel<_Float16>, dim3(blocks), dim3(256), 0, s, w, (_Float16*)out, cout, cin, 0, 0,
                       1.f);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// layer weights [cout][cin][3][3] → packed dgrad conv (cout' = cin, cin' = cout)
int conv3x3_pack_dgrad(const float* w, void* out, int cout, int cin, float scale, int sub2, hipStream_t s) {
    return pack_launch(w, out, cin, cout, 1, sub2, scale, s);
}

}  // namespace isr
