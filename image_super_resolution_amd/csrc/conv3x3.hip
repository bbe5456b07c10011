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

template <int R_, int WM_, int NF_, int KC_, int NST_, int CIN_ = 0, int ABL_ = 0, int PIPE_ = (NF_ == 1), int EPQ_ = 4,
          int SPL_ = 1, int TWN_ = 0>
struct C3 {
    static constexpr int R = R_, WM = WM_, NF = NF_, KC = KC_, NST = NST_;
    static constexpr int PIPE = PIPE_; // 1: double-buffered fragment registers across (k-step, dx) steps
    static constexpr int EPQ = EPQ_;   // epilogue operand units (8 VGPRs each) loaded per pass
    static constexpr int SPL = SPL_;   // the next chunk's LDS-DMA issued in SPL parts, one before each of the first SPL steps
    // tap window: 0 = all 3x3 taps; 1 = taps {0,1}^2; 2 = taps {1,2}^2 (the 2x2 convs that a
    // stride-2 3x3 conv and its transpose become on the 2x2 phase decomposition, isr_conv_desc.taps)
    static constexpr int TWN = TWN_;
    static constexpr int TLO = TWN == 2 ? 1 : 0;
    static constexpr int TN = TWN ? 2 : 3;
    static constexpr int NA = R + TN - 1;  // input rows one wave reads per step
    static constexpr int CIN = CIN_; // 0 = runtime cin; else compile-time (own symbol)
    // Ablation bits, timing-only builds (outputs wrong): 1 = no MFMA (operands
    // kept live), 2 = stage only chunk 0 (no refill), 4 = no epilogue stores.
    // Experiment bits (outputs exact): 8/16 = blocks of the second dispatch round
    // (blockIdx / 256 odd: the second block slot of each CU) start ~0.5/1 us late,
    // so two co-resident blocks are out of phase (one's loads beside the other's MFMAs).
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
    static constexpr int NT = 64 * WM;
    static constexpr int EPS = CT + 4;                 // floats per pixel in the epilogue image
    static constexpr int EP_BYTES = WM * 32 * EPS * 4; // one output row per wave at a time
    static constexpr int LDS = (NST * STAGE > EP_BYTES) ? NST * STAGE : EP_BYTES;
    static constexpr int BPC = 163840 / LDS; // blocks per CU by LDS
    static constexpr int OCC = BPC * WM / 4 >= 2 ? 2 : 1; // waves per SIMD to budget registers for
    static_assert(LDS <= 163840, "LDS budget");
    static_assert(KC == 16 || KC == 32, "chunk width");
};

__device__ __forceinline__ void swap_halves(float& lo, float& hi) {
    // v_permlane32_swap: lanes 32..63 of `lo` trade places with lanes 0..31 of `hi`
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    lo = __uint_as_float(r[0]);
    hi = __uint_as_float(r[1]);
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
template <class C, int MODE>
__device__ __forceinline__ void epilogue(const isr_conv_desc& d, f32x16 (&acc)[C::R][C::NF], int img, int ct,
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
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int g = 0; g < 16; ++g)
                    ep[l31 * EPS + f * 32 + (g & 3) + 8 * (g >> 2) + 4 * hh] = acc[r][f][g];
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
                        *reinterpret_cast<const bf16x8*>(view_at(d.m, img, 2 * yy + si, 2 * x0 + xo, ct * (CT / 4) + cg * 8));
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (!((float)mq[k] > 0.f)) v[k] *= d.mslope;
                }
                if (!(yy < d.h && x0 + xc < d.w)) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = 0.f;
                }
                store8_bf16(view_at(d.y, img, 2 * yy + si, 2 * x0 + xo, ct * (CT / 4) + cg * 8), v);
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
                    if (use_r1) q1[buf][blk] = *reinterpret_cast<const bf16x8*>(view_at(d.r1, img, yy, xx, co));
                }
                if constexpr (MODE & 2) q2[buf][blk] = *reinterpret_cast<const bf16x8*>(view_at(d.r2, img, yy, xx, co));
                if constexpr (MODE & 16) {
                    if (use_m) qm[buf][blk] = *reinterpret_cast<const bf16x8*>(view_at(d.m, img, yy, xx, co));
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
                    if constexpr (MODE & 1) u[e] = u[e] * d.s1 + (use_r1 ? (float)q1[cb][blk][e] : 0.f);
                    if constexpr (MODE & 2) {
                        u[e] = u[e] * d.s2 + (float)q2[cb][blk][e];
                    } else {
                        if (scale2) u[e] *= d.s2;
                    }
                    if constexpr (MODE & 16) {
                        if (use_m && !((float)qm[cb][blk][e] > 0.f)) u[e] *= d.mslope;
                    }
                    if (!valid) u[e] = 0.f;
                }
                const int co = cf + 16 * blk + 8 * hh;
                store8_bf16(view_at(d.y, img, yy, xx, co), u);
                if constexpr (MODE & 4) store8_bf16(view_at(d.y2, img, yy, xx, co), u);
            }
        }
    }
}

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
    if constexpr (C::ABL & 24) {
        if ((blockIdx.x >> 8) & 1) __builtin_amdgcn_s_sleep((C::ABL & 8) ? 16 : 32);
    }

    // ---- per-lane glds source offsets (chunk-invariant) -------------------
    // x_sub2 (backward of PixelShuffle): halo pixel (row, col) of sub-position s
    // lives at x pixel (2row + (s>>1), 2col + (s&1)) — pixel stride 2 plus a
    // per-chunk offset.
    const int ps = d.x_sub2 ? 2 : 1;
    const char* xbase = view_at(d.x, img, ps * (y0 - 1), ps * (x0 - 1), 0);
    const size_t pstride = plane_bytes(d.x);
    const char* wbase = (const char*)d.wpack;
    const int xrow_bytes = d.x.wp * 32;
    auto xchunk = [&](int chunk) -> size_t {
        if (!d.x_sub2) return (size_t)chunk * C::KS * pstride;
        const int cs4 = d.cin >> 2;
        const int c0 = chunk * C::KC;
        const int sp = c0 / cs4, cb = (c0 - sp * cs4) >> 4;
        return (size_t)cb * pstride + (size_t)(sp >> 1) * xrow_bytes + (sp & 1) * 32;
    };
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
                o = (uint32_t)(kp * pstride + ps * (row * xrow_bytes + col * 32) + c * 16);
            }
        } else if (j < C::INSTR) {
            const int u = (j - C::HALO_INSTR) * 64 + lane;
            const int seg = u / (C::CT * 2); // (ks, tap)
            const int rem = u - seg * (C::CT * 2);
            o = (uint32_t)((seg * d.cout + ct * C::CT) * 32 + rem * 16);
        }
        off[k] = o;
    }

    auto stage = [&](int chunk, int buf, int k0 = 0, int k1 = C::IPW) {
        char* dst = smem + buf * C::STAGE;
        const char* xs = xbase + xchunk(chunk);
        const char* ws = wbase + (size_t)chunk * wchunk_bytes;
#pragma unroll
        for (int k = k0; k < k1; ++k) {
            const int j = wave + WM * k;
            const char* src = (j < C::HALO_INSTR ? xs : ws) + off[k];
            glds16(src, dst + j * 1024);
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
        const bool refill = !(C::ABL & 2) && chunk + C::NST - 1 < nchunks;
        if constexpr (C::SPL <= 1) {
            if (refill) stage(chunk + C::NST - 1, (chunk + C::NST - 1) % C::NST);
        }

        const char* hs = smem + ((C::ABL & 2) ? 0 : (chunk % C::NST)) * C::STAGE;
        const char* ws = hs + C::HALO_INSTR * 1024;
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
                if constexpr (C::ABL & 32) {
                    // timing probe: dx > TLO fragments = previous dx's shifted one lane by DPP
                    // (lanes 31/63 not fixed up: outputs wrong)
                    if (st % TN != 0) {
                        const int prev = C::PIPE ? set ^ 1 : set;
                        auto* src = reinterpret_cast<int*>(&fa[prev][ia]);
                        auto* dst = reinterpret_cast<int*>(&fa[set][ia]);
#pragma unroll
                        for (int e = 0; e < 4; ++e) dst[e] = __builtin_amdgcn_update_dpp(0, src[e], 0x130, 0xf, 0xf, false);
                        continue;
                    }
                }
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
                const int q = qw + (TLO + ia) * C::HC + dx;
                fa[set][ia] = lds_read16(hs + ks * C::HIPL * 1024 + halo_unit2(q, hh) * 16);
            }
        };
        if constexpr (C::PIPE) load_step(0, 0);
        if constexpr (C::PIPE == 2) __builtin_amdgcn_sched_barrier(0);
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
                for (int ia = 0; ia < NA; ++ia)
#pragma unroll
                    for (int dyi = 0; dyi < TN; ++dyi) {
                        const int r = ia - dyi;
                        if (r >= 0 && r < R) {
#pragma unroll
                            for (int f = 0; f < NF; ++f) {
                                acc[r][f] = mfma32(fb[cur][dyi][f], fa[cur][ia], acc[r][f]);
                                if (st + 1 < NS)
                                    for (int k = m * NRD / NM; k < (m + 1) * NRD / NM; ++k) read_one(st + 1, k, cur ^ 1);
                                __builtin_amdgcn_sched_barrier(0);  // pin the (MFMA, reads) order
                                ++m;
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
                            } else if constexpr (C::ABL & 64) {
                                // DVFS probe (outputs wrong): the same FLOPs as two 16x16x32 MFMAs
                                f32x16& a = acc[r][f];
                                const int h = (r + f) & 1;
                                f32x4 c0 = {a[8 * h], a[8 * h + 1], a[8 * h + 2], a[8 * h + 3]};
                                f32x4 c1 = {a[8 * h + 4], a[8 * h + 5], a[8 * h + 6], a[8 * h + 7]};
                                c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][dyi][f], fa[cur][ia], c0, 0, 0, 0);
                                c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][dyi][f], fa[cur][ia], c1, 0, 0, 0);
#pragma unroll
                                for (int e = 0; e < 4; ++e) { a[8 * h + e] = c0[e]; a[8 * h + 4 + e] = c1[e]; }
                            } else {
                                acc[r][f] = mfma32(fb[cur][dyi][f], fa[cur][ia], acc[r][f]);
                            }
                        }
                    }
                }
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier(); // all waves done reading the ring before it becomes the epilogue image

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
                                    : ((d.r1.data ? 1 : 0) | (d.r2.data ? 2 : 0) | (d.y2.data ? 4 : 0) | (d.m.data ? 16 : 0));
    switch (mode) {
        case 0: epilogue<C, 0>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 1: epilogue<C, 1>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 2: epilogue<C, 2>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 3: epilogue<C, 3>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 4: epilogue<C, 4>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 5: epilogue<C, 5>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 6: epilogue<C, 6>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 7: epilogue<C, 7>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 8: epilogue<C, 8>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 24: epilogue<C, 24>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 16: epilogue<C, 16>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 17: epilogue<C, 17>(d, acc, img, ct, x0, y0, wave, lane); break;
        case 18: epilogue<C, 18>(d, acc, img, ct, x0, y0, wave, lane); break;
        default: epilogue<C, 19>(d, acc, img, ct, x0, y0, wave, lane); break;  // 19; y2 + mask is rejected by isr_conv3x3_fwd
    }
}

template <class C>
static int launch3x3(const isr_conv_desc* d, hipStream_t s) {
    if (d->cout % C::CT || d->cin % C::KC || d->ha % C::TH) return -2;
    if (C::CIN && d->cin != C::CIN) return -2;
    auto kern = conv3x3_fwd_kernel<C>;
    lds_limit((const void*)kern, C::LDS);
    const int blocks = (d->wa / C::TW) * (d->ha / C::TH) * d->n * (d->cout / C::CT);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(C::NT), C::LDS, s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Variant table: variant 0 is the production choice per shape; the others are
// kept for on-device A/B tuning (isr_conv3x3_fwd_variant, tools/tune_conv.py).
// (tools/tune_conv.py on MI355X, N=16 128²: the 16x32-tile, 2-blocks/CU configs are
// fastest on every shape of the generator; the 32x32 8-wave tiles win only at long K)
// cout == 32 (RDB growth convs)
// V_G0 / V_F0: the next step's fragment reads interleaved one per MFMA (PIPE 2): 2-7 % over the
// batched prefetch, whose 18-24 reads in flight exceed lgkmcnt's range (so hipcc waited lgkmcnt(0))
using V_G0 = C3<4, 4, 1, 16, 2, 0, 0, 2>; // 16x32, 4 waves, KC16 double buffer, 64 KB → 2 blocks / CU
using V_G1 = C3<4, 8, 1, 16, 3>; // 32x32 px tile, 8 waves, 3-deep KC16 ring
using V_G2 = C3<2, 4, 1, 32, 2>; // 8x32, KC32, 2 blocks / CU
using V_G3 = C3<2, 8, 1, 16, 3>; // 16x32, 8 waves x 2 rows, 3-deep KC16 ring
// cout % 64 == 0
using V_W0 = C3<4, 4, 2, 16, 2, 0, 0, 2>; // 16x32, 4 waves, KC16 double buffer, 80 KB → 2 blocks / CU, PIPE 2
using V_W1 = C3<4, 8, 2, 16, 2>; // 32x32 px tile, 8 waves, KC16 double buffer
using V_W2 = C3<2, 4, 2, 32, 2>; // 8x32, KC32
using V_W3 = C3<4, 4, 2, 32, 2>; // 16x32, KC32, 1 block / CU
using V_F0 = C3<4, 4, 2, 16, 2, 192, 0, 2>; // RDB final conv 192→64: V_W0 with compile-time cin, PIPE 2

int conv3x3_fwd_variant(const isr_conv_desc* d, int variant, hipStream_t s) {
    if (d->cout % 64) {  // 32-cout tiles: growth convs (cout 32) and dgrad of them (96, 160)
        switch (variant) {
            case 0: return launch3x3<V_G0>(d, s);
            case 1: return launch3x3<V_G1>(d, s);
            case 2: return launch3x3<V_G2>(d, s);
            case 3: return launch3x3<V_G3>(d, s);
#ifdef ISR_TUNING
            // ablations of V_G0 (timing only, outputs wrong): tuning builds only
            case 4: return launch3x3<C3<4, 4, 1, 16, 2, 0, 1>>(d, s);
            case 5: return launch3x3<C3<4, 4, 1, 16, 2, 0, 2>>(d, s);
            case 6: return launch3x3<C3<4, 4, 1, 16, 2, 0, 4>>(d, s);
            case 7: return launch3x3<C3<4, 4, 1, 16, 2, 0, 3>>(d, s);
            case 16: return launch3x3<C3<4, 4, 1, 16, 2, 0, 32>>(d, s);  // probe: dx>0 activations by DPP shift
            case 20: return launch3x3<C3<4, 4, 1, 16, 2, 0, 64>>(d, s);  // DVFS probe: 2x 16x16x32 per 32x32x16
#endif
            case 8: return launch3x3<C3<4, 4, 1, 16, 2, 0, 0, 1, 1>>(d, s);  // V_G0, one unit per epilogue pass
            case 9: return launch3x3<C3<4, 4, 1, 16, 2, 0, 0, 1, 4, 2>>(d, s);  // V_G0, refill split over 2 steps
            case 10: return launch3x3<C3<4, 4, 1, 16, 2, 0, 0, 1, 4, 3>>(d, s); // V_G0, refill split over 3 steps
            case 11: return launch3x3<C3<2, 4, 1, 16, 3>>(d, s);  // 8x32 tile, 3-deep ring (60 KB, 2 blocks/CU)
            case 12: return launch3x3<C3<4, 4, 1, 16, 3>>(d, s);  // 16x32 tile, 3-deep ring (1 block/CU)
            case 13: return launch3x3<C3<2, 4, 1, 16, 2>>(d, s);  // 8x32 tile, double buffer (3 blocks/CU)
            case 14: return launch3x3<C3<4, 4, 1, 16, 2, 0, 8>>(d, s);   // V_G0, second block slot ~0.5 us late
            case 15: return launch3x3<C3<4, 4, 1, 16, 2, 0, 16>>(d, s);  // V_G0, second block slot ~1 us late
            case 17: return launch3x3<C3<4, 4, 1, 16, 2, 0, 0, 2>>(d, s);  // V_G0, reads interleaved with MFMAs
            case 18: return launch3x3<C3<4, 4, 1, 32, 2, 0, 0, 2>>(d, s);  // KC32 (1 block/CU), interleaved
            case 19: return launch3x3<C3<2, 4, 1, 32, 2, 0, 0, 2>>(d, s);  // 8x32 KC32, interleaved
            case 21: return launch3x3<C3<8, 4, 1, 16, 2, 0, 0, 2>>(d, s);  // 32x32 tile, 8 rows per wave (1 block/CU)
            case 22: return launch3x3<C3<8, 2, 1, 16, 2, 0, 0, 2>>(d, s);  // 16x32 tile, 2 waves x 8 rows
            case 23: return launch3x3<C3<2, 8, 1, 16, 2, 0, 0, 2>>(d, s);  // 16x32 tile, 8 waves x 2 rows
            case 24: return launch3x3<C3<2, 4, 1, 16, 2, 0, 0, 2>>(d, s);  // 8x32 tile, double buffer, interleaved
            case 25: return launch3x3<C3<2, 4, 1, 16, 3, 0, 0, 2>>(d, s);  // 8x32 tile, 3-deep ring, interleaved
        }
        return -2;
    }
    switch (variant) {
        case 0: return d->cin == 192 ? launch3x3<V_F0>(d, s) : launch3x3<V_W0>(d, s);
        case 1: return launch3x3<V_W1>(d, s);
        case 2: return launch3x3<V_W2>(d, s);
        case 3: return launch3x3<V_W3>(d, s);
#ifdef ISR_TUNING
        // ablations of V_W0 (timing only, outputs wrong): tuning builds only
        case 4: return launch3x3<C3<4, 4, 2, 16, 2, 0, 1>>(d, s);
        case 5: return launch3x3<C3<4, 4, 2, 16, 2, 0, 2>>(d, s);
        case 6: return launch3x3<C3<4, 4, 2, 16, 2, 0, 4>>(d, s);
        case 7: return launch3x3<C3<4, 4, 2, 16, 2, 0, 3>>(d, s);
        case 16: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 32>>(d, s)  // probe: DPP-shifted dx>0
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 32>>(d, s);
        case 20: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 64>>(d, s)  // DVFS probe (16x16x32)
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 64>>(d, s);
#endif
        case 8: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 0, 0, 1>>(d, s)  // V_F0 / V_W0, one unit per pass
                                     : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 0, 1>>(d, s);
        case 9: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 0, 0, 4, 2>>(d, s)  // refill split over 2 steps
                                     : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 0, 4, 2>>(d, s);
        case 10: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 0, 1, 4, 1>>(d, s)  // pipelined fragment reads
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 1, 4, 1>>(d, s);
        case 11: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 0, 1, 4, 2>>(d, s)  // both
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 1, 4, 2>>(d, s);
        case 14: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 8>>(d, s)  // second block slot ~0.5 us late
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 8>>(d, s);
        case 15: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 16>>(d, s)  // ~1 us late
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 16>>(d, s);
        case 17: return d->cin == 192 ? launch3x3<C3<4, 4, 2, 16, 2, 192, 0, 2>>(d, s)  // reads interleaved with MFMAs
                                      : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 2>>(d, s);
        case 18: return d->cin == 192 ? launch3x3<C3<2, 4, 2, 32, 2, 192, 0, 2>>(d, s)  // 8x32 KC32, interleaved
                                      : launch3x3<C3<2, 4, 2, 32, 2, 0, 0, 2>>(d, s);
        case 24: return d->cin == 192 ? launch3x3<C3<2, 4, 2, 16, 2, 192, 0, 2>>(d, s)  // 8x32 tile, interleaved
                                      : launch3x3<C3<2, 4, 2, 16, 2, 0, 0, 2>>(d, s);
    }
    return -2;
}

int conv3x3_fwd_dispatch(const isr_conv_desc* d, hipStream_t s) {
    if (d->taps == 1) return d->cout % 64 ? -2 : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 0, 4, 1, 1>>(d, s);
    if (d->taps == 2) return d->cout % 64 ? -2 : launch3x3<C3<4, 4, 2, 16, 2, 0, 0, 0, 4, 1, 2>>(d, s);
    return conv3x3_fwd_variant(d, 0, s);
}

// ---- weight packing: fp32 OIHW → bf16 [c16][tap][cout][hpos][8] -----------
// Forward: the packed conv has (cout, cin) = the layer's, element W[n][ci][tap].
// dgrad (transposed): the packed conv maps the layer's output gradient (cin' =
// layer cout) to its input gradient (cout' = layer cin): element
// scale * W[co(ci')][n][8 - tap] (180° rotation), where with sub2 the input
// channel ci' = s*(layer cout/4) + c stands for layer channel co = 4c + s
// (PixelShuffle order, see isr_conv_desc.x_sub2).
__device__ __forceinline__ void pack3x3_range(const float* __restrict__ w, __bf16* __restrict__ out, int pcout,
                                              int pcin, int transposed, int sub2, float scale, size_t first,
                                              size_t stride) {
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
            v = w[((size_t)co * pcout + n) * 9 + (8 - tap)];       // layer W[co][n][8 - tap]; layer cin = pcout
        }
        out[idx] = (__bf16)(v * scale);
    }
}

__global__ void pack3x3_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int pcout, int pcin,
                               int transposed, int sub2, float scale) {
    pack3x3_range(w, out, pcout, pcin, transposed, sub2, scale, blockIdx.x * (size_t)blockDim.x + threadIdx.x,
                  (size_t)gridDim.x * blockDim.x);
}

// Many packs in one launch (the training plan repacks every conv each step):
// blockIdx.y = item, blockIdx.x strides over that item's elements.
__global__ void pack3x3_batch_kernel(const isr_pack_item* __restrict__ items) {
    const isr_pack_item it = items[blockIdx.y];
    const int pcout = it.dgrad ? it.cin : it.cout, pcin = it.dgrad ? it.cout : it.cin;
    pack3x3_range(it.w, (__bf16*)it.out, pcout, pcin, it.dgrad, it.sub2, it.dgrad ? it.scale : 1.f,
                  blockIdx.x * (size_t)blockDim.x + threadIdx.x, (size_t)gridDim.x * blockDim.x);
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
    hipLaunchKernelGGL(pack3x3_kernel, dim3(blocks), dim3(256), 0, s, w, (__bf16*)out, pcout, pcin, transposed, sub2,
                       scale);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int conv3x3_pack(const float* w, void* out, int cout, int cin, hipStream_t s) {
    return pack_launch(w, out, cout, cin, 0, 0, 1.f, s);
}

// layer weights [cout][cin][3][3] → packed dgrad conv (cout' = cin, cin' = cout)
int conv3x3_pack_dgrad(const float* w, void* out, int cout, int cin, float scale, int sub2, hipStream_t s) {
    return pack_launch(w, out, cin, cout, 1, sub2, scale, s);
}

}  // namespace isr
