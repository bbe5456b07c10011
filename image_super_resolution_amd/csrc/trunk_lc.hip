// The RRDB trunk (utils/models.py:298-317 RRDB.forward over :245-271 RDB.forward) as ONE persistent
// launch in the loader / consumer form (isr_conv_chain variant 9).
//
// Why.  The pair form (trunk.hip) makes every computing wave stage its own share of the LDS ring:
// per 16-channel K-chunk each wave waits for its DMA, passes a workgroup barrier and issues 7-11
// LDS-DMA pieces (~200 cycles of wave time each, tuning ablations round 4) around 36 (growth) /
// 72 (final) MFMAs of its own — 7,900-11,700 cycles per chunk against 1,152 / 2,304 cycles of
// matrix work (profiles/r04_trunk_items_pair.jsonl), MFMA busy 0.54.  Here the roles split
// (cdna_hip_programming.md / megakernel ring: FULL / FREE words in LDS):
//  * ONE 8-wave workgroup per CU: waves 0-3 compute (4 output rows x 32 px each: the pair form's
//    16 x 32 tile and its MFMA order), waves 4-7 only load (one of each per SIMD);
//  * a 4-slot LDS ring (38 KB slots: one chunk's 18 x 34 halo plane + its 32 / 64-cout weights),
//    the loaders keeping up to 3 chunks in flight; per slot a FULL count (+1 per loader wave once
//    its pieces of the chunk have landed: counted vmcnt) and a FREE count (+1 per compute wave
//    once it has issued its last LDS read of the chunk);
//  * the compute waves never issue LDS-DMA, never pass a barrier inside the trunk and never poll
//    another workgroup: they wait for FULL, read fragments, run the MFMAs, signal FREE;
//  * the loaders do the tile-neighbourhood dependency polls (before staging the first chunk the
//    previous layer wrote, as trunk.hip) after handing every landed chunk to the consumers, so a
//    blocked loader never holds back work its own compute waves could finish;
//  * a tile's outputs (sc1 write-through stores, Guideline 16 R1) are published by the LAST of the
//    four compute waves to drain its stores (an LDS counter, no barrier), with the same relaxed
//    agent-scope progress word gen * 1024 + L + 1 as trunk.hip.
// The MFMA order per accumulator is the pair form's (kernel-row-major, residual fold between the
// dy = 1 and dy = 2 contributions of chunks 0-3), so the outputs equal the per-conv launches bit
// for bit (tests/test_gpu_chain.py).
#include "trunk_common.h"

namespace isr {

// An A/B form: bitwise equal to the per-conv launches, but 1-3 % SLOWER than the pair form on the
// bench forward — compiled into the tuning library only.
#ifdef ISR_TUNING

namespace lc {
constexpr int WMC = 4;                          // compute waves
constexpr int WML = 4;                          // loader waves
constexpr int NT = 64 * (WMC + WML);
constexpr int R = 4, TH = 16, TN = 3, NA = R + 2;
constexpr int HQ = (TH + 2) * tk::HC;           // 612 halo pixels per chunk
constexpr int HP = (HQ + 31) / 32;              // 20 halo pieces (1 KB)
constexpr int SLOT = (HP + tk::WPF) * 1024;     // 38,912 B: halo + 64-cout weights
constexpr int NS = 4;                           // ring slots
constexpr int INFL = 3;                         // chunks a loader keeps in flight (< NS)
constexpr int BIAS_OFF = NS * SLOT;             // 4 bias slots of 256 B
constexpr int FLAG_OFF = BIAS_OFF + 4 * 256;    // FULL[NS], FREE[NS], DONE (u32 each)
constexpr int LDS = FLAG_OFF + 64;
constexpr int HPW = (HP + WML - 1) / WML;       // halo pieces per loader wave (5)
constexpr int WPW = (tk::WPF + WML - 1) / WML;  // weight pieces per loader wave (<= 5)
static_assert(LDS <= 163840, "LDS budget");
static_assert(INFL < NS, "a loader never waits for a slot whose chunk it has not handed over");
}  // namespace lc

// Tuning builds: ablation bits (timing only, outputs wrong): 1 = loaders skip the halo DMA, 8 = the
// weight DMA, 16 = the dependency waits; 2 = compute waves skip fragment reads and MFMAs, 4 = the
// epilogue stores.
#ifdef ISR_TUNING
__device__ int g_lc_knobs[4];
__device__ __forceinline__ int lc_abl_load() { return __builtin_amdgcn_readfirstlane(g_lc_knobs[0]); }
int trunk_lc_knobs_set(const int* k) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_lc_knobs), k, 4 * sizeof(int)) == hipSuccess ? 0 : -1;
}
#else
__device__ __forceinline__ int lc_abl_load() { return 0; }
#endif

struct LcArgs {
    unsigned* state;
    int rec_off;   // words
    int nl;
    int acquire;
};

struct LcCtx {
    unsigned* state;
    unsigned gen;
    int acquire;
    int hp, wp, cs16, pad, h, w, nbx, nby, ntiles;
    uint32_t pstride;  // bytes per 16-channel plane (< 2 GiB): each buffer resource spans one
    int abl;           // tuning ablation bits (0 in production builds)
};

// ---- LDS words (flags) -------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(int off) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    return (uint32_t)(uintptr_t)ISR_LDS_PTR(smem + off);
}

__device__ __forceinline__ unsigned lds_word(int off) {
    unsigned v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(off)) : "memory");
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ void lds_inc(int off) {  // one lane of the calling wave adds 1
    if ((threadIdx.x & 63) == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(lds_addr(off)), "v"(1u) : "memory");
}

__device__ __forceinline__ unsigned lds_inc_rtn(int off) {  // lane 0 adds 1; the old value, uniform
    unsigned v = 0;
    if ((threadIdx.x & 63) == 0)
        asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(off)), "v"(1u) : "memory");
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ void lc_give_up(const LcCtx& c) {
    if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store(c.state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(c.state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Wait until the LDS count at `off` reaches `target` (serial arithmetic).  Bounded: a launch that
// gave up anywhere (state[1] == gen) stops waiting, so the grid always drains.
__device__ __forceinline__ void lds_wait_ge(const LcCtx& c, int off, unsigned target) {
    for (unsigned spins = 0;; ++spins) {
        if ((int)(lds_word(off) - target) >= 0) return;
        if ((spins & 255) == 255 &&
            __hip_atomic_load(c.state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c.gen)
            return;
        if (spins > (1u << 22)) {
            lc_give_up(c);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ int lc_full(int slot) { return lc::FLAG_OFF + 4 * slot; }
__device__ __forceinline__ int lc_free(int slot) { return lc::FLAG_OFF + 16 + 4 * slot; }
constexpr int LC_DONE = lc::FLAG_OFF + 32;

// ---- loader waves --------------------------------------------------------------------------
// The loaders walk the same (layer, tile, chunk) stream as the compute waves.  Loader wave lw
// issues halo pieces lw, lw + 4, ... (< 20), weight pieces lw, lw + 4, ... (< 9 / 18), and (lw 0)
// the tile's bias with its chunk 0.  `pend` chunks issued but not yet handed over (FULL) by
// this wave: their slots and vmcnt marks in a 3-deep FIFO of named scalars.
struct LcPend {
    int n;
    int s0, s1, s2;          // slots, oldest first
    uint32_t m0, m1, m2;     // `issued` right after each chunk's pieces
};

__device__ __forceinline__ void lc_hand_oldest(LcPend& p, uint32_t issued) {
    wait_vm(issued - p.m0);
    lds_inc(lc_full(p.s0));
    p.s0 = p.s1;
    p.s1 = p.s2;
    p.m0 = p.m1;
    p.m1 = p.m2;
    --p.n;
}

__device__ __forceinline__ void lc_hand_all(LcPend& p) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (p.n > 0) lds_inc(lc_full(p.s0));
    if (p.n > 1) lds_inc(lc_full(p.s1));
    if (p.n > 2) lds_inc(lc_full(p.s2));
    p.n = 0;
}

// forceinline: as an outlined call its context went through scratch, and scratch loads counted in
// vmcnt would weaken the counted waits that hand chunks to the consumers
__device__ __forceinline__ void lc_loader(const LcCtx& c, const_rec* recs, int nl, int G, int b, int lw) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    uint32_t hoff[lc::HPW];
#pragma unroll
    for (int k = 0; k < lc::HPW; ++k) hoff[k] = halo_piece_off<lc::HQ>(lw + lc::WML * k, lane, c.wp);
    uint32_t issued = 0;
    LcPend p;
    p.n = 0;
    p.s0 = p.s1 = p.s2 = 0;
    p.m0 = p.m1 = p.m2 = 0;
    unsigned item = 0;
    int tseq = 0;
    for (int L = 0; L < nl; ++L) {
        const_rec& rec = recs[L];
        const int nch = rec_nch(rec), first_new = rec_first_new(rec);
        const int wpc = rec_kind(rec) == 1 ? tk::WPF : tk::WPG;
        const uint32_t wbytes = (uint32_t)(nch * wpc * 1024);
        const auto rw = rsrc_n((const void*)(uintptr_t)rec.w, wbytes);
        const unsigned need = c.gen * 1024u + (unsigned)L;
        for (int t = b; t < c.ntiles; t += G, ++tseq) {
            const int bx = t % c.nbx, tmp = t / c.nbx, by = tmp % c.nby, img = tmp / c.nby;
            const char* xbase = (const char*)(uintptr_t)rec.x +
                                (size_t)((uint32_t)img * c.cs16 + rec_xp(rec)) * c.pstride;
            const uint32_t h0 = (uint32_t)(((by * lc::TH - 1 + c.pad) * c.wp + (bx * tk::TW - 1 + c.pad)) * 32);
            bool dep_ok = first_new == tk::NEED_NONE;
            for (int ch = 0; ch < nch; ++ch, ++item) {
                const int slot = (int)(item % lc::NS);
                if (item >= (unsigned)lc::NS) {  // the slot's previous chunk consumed by every compute wave
                    const unsigned tgt = 4u * (item / lc::NS);
                    if ((int)(lds_word(lc_free(slot)) - tgt) < 0) lds_wait_ge(c, lc_free(slot), tgt);
                }
                if (!dep_ok && ch >= first_new && !(c.abl & 16)) {
                    // every landed chunk goes to the consumers first: the neighbourhood may be
                    // waiting for this workgroup's own tiles
                    lc_hand_all(p);
                    dep_wait(c.state, nb_of(t, c.nbx, c.nby), need, c.gen);
                    if (c.acquire) acquire_fence();
                    dep_ok = true;
                }
                char* dst = smem + slot * lc::SLOT;
                const auto rx = rsrc_n(xbase + (size_t)ch * c.pstride, c.pstride);
#pragma unroll
                for (int k = 0; k < lc::HPW; ++k) {
                    const int j = lw + lc::WML * k;
                    if (j < lc::HP && !(c.abl & 1)) {
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, ISR_LDS_PTR(dst + j * 1024), 16, hoff[k], h0, 0, 16);
                        ++issued;
                    }
                }
                const uint32_t wo = (uint32_t)(ch * wpc * 1024);
#pragma unroll
                for (int k = 0; k < lc::WPW; ++k) {
                    const int j = lw + lc::WML * k;
                    if (j < wpc && !(c.abl & 8)) {
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, ISR_LDS_PTR(dst + (lc::HP + j) * 1024), 16,
                                                                 lane * 16, wo + j * 1024, 0, 0);
                        ++issued;
                    }
                }
                if (ch == 0 && lw == 0) {
                    if (lane < (wpc == tk::WPG ? 32 : 64))  // cout floats only
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            rsrc_n((const void*)(uintptr_t)rec.b, wpc == tk::WPG ? 128u : 256u),
                            ISR_LDS_PTR(smem + lc::BIAS_OFF + (tseq & 3) * 256), 4, lane * 4, 0, 0, 0);
                    ++issued;
                }
                // FIFO push, then hand over the oldest chunks beyond INFL - 1 still pending
                if (p.n == 0) { p.s0 = slot; p.m0 = issued; }
                else if (p.n == 1) { p.s1 = slot; p.m1 = issued; }
                else { p.s2 = slot; p.m2 = issued; }
                ++p.n;
                if (p.n >= lc::INFL) lc_hand_oldest(p, issued);
            }
        }
    }
    lc_hand_all(p);
}

// ---- compute waves -------------------------------------------------------------------------
// A finished tile whose progress word is not yet published (its stores are drained later, behind
// the next tile's first chunk, instead of stalling the matrix pipe right after the epilogue).
struct LcPub {
    bool pend;
    int t, tseq;
    unsigned v;
};

__device__ __forceinline__ void lc_publish(const LcCtx& c, LcPub& pb) {
    if (!pb.pend) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have landed
    if (lds_inc_rtn(LC_DONE) == 4u * (unsigned)pb.tseq + 3u && (threadIdx.x & 63) == 0)  // the last wave
        __hip_atomic_store(c.state + 4 + pb.t, pb.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pb.pend = false;
}

template <int NF, bool MASKED>
__device__ __forceinline__ void lc_tile(const LcCtx& c, unsigned& item, LcPub& pb, int tseq, const_rec& rec, int L,
                                        int t, int wave) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = lc::R, TN = lc::TN, NA = lc::NA, CT = 32 * NF;
    const int lane = threadIdx.x & 63, l31 = lane & 31, hh = lane >> 5;
    const int bx = t % c.nbx, tmp = t / c.nbx, by = tmp % c.nby, img = tmp / c.nby;
    const int x0 = bx * tk::TW, y0 = by * lc::TH;
    const int nch = rec_nch(rec);
    const bool fold = NF == 2 && rec_fold(rec);
    const bool has_r2 = NF == 2 && rec.r2 != 0;
    constexpr bool masked = NF == 1 && MASKED;
    const int bslot = tseq & 3;
    const uint32_t a_w = (uint32_t)(lc::HP * 1024 + (2 * l31 + (hh ^ ((l31 >> 3) & 1))) * 16);
    uint32_t a_h[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
        a_h[dx] = (uint32_t)((wave * R * tk::HC + l31 + dx) * 32 + 16 * (hh ^ (((l31 + dx) >> 3) & 1)));
    const uint32_t idv = rec_idv(rec);
    f32x16 acc[R][NF];
    // two fragment sets: chunk ch computes step s from set (s + ch) & 1, so during its step 2 the
    // other set is free for the NEXT chunk's step-0 fragments (read there when that chunk's slot
    // is already full: no exposed read latency and no FULL wait at the next chunk's top)
    bf16x8 fb[2][TN][NF], fa[2][NA];
    auto read_one = [&](const char* sb, int dx, int idx, int set) {
        if (idx < TN * NF) {
            const int dyi = idx / NF, f = idx % NF;
            fb[set][dyi][f] = lds_read16(sb + a_w + ((dyi * 3 + dx) * CT * 2 + f * 64) * 16);
        } else {
            const int ia = idx - TN * NF;
            fa[set][ia] = lds_read16(sb + a_h[dx] + ia * tk::HC * 32);
        }
    };
    // step 0's q-th fragment in order of first use (kernel-row-major MFMA order): kernel row 0's
    // weights, input rows 0..R-1, kernel row 1's weights, row R, kernel row 2's weights, row R+1
    constexpr int NS0 = TN * NF + NA;
    auto read_s0 = [&](const char* sb, int q, int set) {
        if (q < NF) read_one(sb, 0, q, set);
        else if (q < NF + R) read_one(sb, 0, TN * NF + (q - NF), set);
        else if (q < 2 * NF + R) read_one(sb, 0, NF + (q - NF - R), set);
        else if (q == 2 * NF + R) read_one(sb, 0, TN * NF + R, set);
        else if (q < 3 * NF + R + 1) read_one(sb, 0, 2 * NF + (q - 2 * NF - R - 1), set);
        else read_one(sb, 0, TN * NF + R + 1, set);
    };
    bool pf = false;  // the current chunk's step-0 fragments were read by the previous chunk
    // the previous tile's publish, as plain locals: a struct reference live across the inline-asm
    // waits here was kept in memory by hipcc (scratch spills around every chunk)
    bool ppend = pb.pend;
    const int pt = pb.t, ptseq = pb.tseq;
    const unsigned pv = pb.v;
    auto publish_prev = [&]() {
        if (!ppend) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lds_inc_rtn(LC_DONE) == 4u * (unsigned)ptseq + 3u && (threadIdx.x & 63) == 0)
            __hip_atomic_store(c.state + 4 + pt, pv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ppend = false;
    };

    auto do_chunk = [&](const int ch, auto fc_tag, auto p_tag) {
        constexpr int FC = decltype(fc_tag)::value, P = decltype(p_tag)::value;
        const int slot = (int)(item % lc::NS);
        const char* sb = smem + slot * lc::SLOT;
        if (!pf) {
            const unsigned tgt = 4u * (item / lc::NS + 1);
            if (ppend && (int)(lds_word(lc_full(slot)) - tgt) < 0) publish_prev();  // never wait holding it
            lds_wait_ge(c, lc_full(slot), tgt);
            if (ch == 0) {  // bias -> accumulators (register g of lane l: cout (g&3) + 8(g>>2) + 4hh)
                const float* bs = reinterpret_cast<const float*>(smem + lc::BIAS_OFF + bslot * 256);
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    f32x16 b0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const f32x4 q = *reinterpret_cast<const f32x4*>(bs + f * 32 + 8 * j + 4 * hh);
#pragma unroll
                        for (int e = 0; e < 4; ++e) b0[4 * j + e] = q[e];
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[r][f] = b0;
                }
            }
            if (c.abl & 2) {  // tuning ablation: no fragment reads, no MFMAs
                lds_inc(lc_free(slot));
                ++item;
                return;
            }
#pragma unroll
            for (int q = 0; q < NS0; ++q) read_s0(sb, q, P);
            __builtin_amdgcn_sched_barrier(0);
        }
        pf = false;
        __builtin_amdgcn_s_setprio(1);
        // MFMAs: 3 steps (dx), each kernel-row-major (dy, then output row r) — every accumulator
        // sees dy 0, 1, 2 in that order, as in trunk.hip and conv3x3.hip (bit-identical sums)
#pragma unroll
        for (int stp = 0; stp < 3; ++stp) {
            const int cur = (stp + P) & 1;
            bool pre = false;
            const char* nsb = sb;
            if (stp == 2) {
                // every LDS read of this slot has been issued (step 2's fragments were read during
                // step 1): LDS executes a wave's ops in order, so the slot may be refilled now
                lds_inc(lc_free(slot));
                // the next slot's step-0 fragments are read below in any case (unconditional reads
                // keep the free set's old values dead); they count only when that chunk belongs to
                // this tile and its slot was already full here
                const int nslot = (int)((item + 1) % lc::NS);
                nsb = smem + nslot * lc::SLOT;
                pre = ch + 1 < nch && (int)(lds_word(lc_full(nslot)) - 4u * ((item + 1) / lc::NS + 1)) >= 0;
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int dyi = 0; dyi < TN; ++dyi) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
#pragma unroll
                    for (int f = 0; f < NF; ++f) acc[r][f] = mfma32(fb[cur][dyi][f], fa[cur][r + dyi], acc[r][f]);
                    if constexpr (NF == 2 && FC >= 0) {
                        if (dyi == 1 && stp == 1) {  // residual fold: + x/s1 on the centre pixels of row r
                            const bf16x8 a = fold_a_bits<false>(idv, FC & 1);
                            acc[r][FC >> 1] = mfma32(a, fa[cur][r + 1], acc[r][FC >> 1]);
                        }
                    }
                    if (stp + 1 < 3 && (dyi == 2 || r == 0)) read_one(sb, stp + 1, TN * NF + r + dyi, cur ^ 1);
                    if (stp == 2 && dyi * R + r < NS0) read_s0(nsb, dyi * R + r, cur ^ 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (stp + 1 < 3) {
#pragma unroll
                    for (int f = 0; f < NF; ++f) read_one(sb, stp + 1, dyi * NF + f, cur ^ 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (stp == 2) pf = pre;
        }
        __builtin_amdgcn_s_setprio(0);
        ++item;
        publish_prev();  // the previous tile's stores are long done by now
    };
    int ch0 = 0;
    if constexpr (NF == 2) {
        if (fold && nch >= 4) {
            do_chunk(0, TIC<0>{}, TIC<0>{});
            do_chunk(1, TIC<1>{}, TIC<1>{});
            do_chunk(2, TIC<2>{}, TIC<0>{});
            do_chunk(3, TIC<3>{}, TIC<1>{});
            ch0 = 4;
        }
    }
    for (int ch = ch0; ch < nch; ch += 2) {  // chunk parity = ch & 1 (compile-time set indices; nch even)
        do_chunk(ch, TIC<-1>{}, TIC<0>{});
        do_chunk(ch + 1, TIC<-1>{}, TIC<1>{});
    }

    // ---- epilogue: straight from the accumulators, write-through (sc1) stores (trunk.hip) ----
    {
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const int xx = x0 + l31;
        const float slope = rec.slope, s1 = rec.s1, s2 = rec.s2;
        const bool scale2 = s2 != 1.f;
        const char* ybase = (const char*)(uintptr_t)rec.y + (size_t)((uint32_t)img * c.cs16 + rec_yp(rec)) * c.pstride;
        bf16x8 q2[R][NF][2];
        const char* r2base = (const char*)(uintptr_t)rec.r2 + (size_t)((uint32_t)img * c.cs16 + rec_r2p(rec)) * c.pstride;
        auto load_r2 = [&](int r) {
            const uint32_t pix = (uint32_t)((y0 + wave * R + r + c.pad) * c.wp + xx + c.pad);
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const auto rr = rsrc_n(r2base + (size_t)(2 * f + blk) * c.pstride, c.pstride);
                    q2[r][f][blk] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rr, pix * 32 + 16 * hh, 0, 16));
                }
        };
        if (has_r2 || masked) load_r2(0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((has_r2 || masked) && r + 1 < R) load_r2(r + 1);
            const int yy = y0 + wave * R + r;
            const bool valid = yy < c.h && xx < c.w;
            const uint32_t pix = (uint32_t)((yy + c.pad) * c.wp + xx + c.pad);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                float v[16];
#pragma unroll
                for (int g = 0; g < 16; ++g) v[g] = acc[r][f][g];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    swap_halves(v[k], v[4 + k]);
                    swap_halves(v[8 + k], v[12 + k]);
                }
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    float* u = v + 8 * blk;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        if (masked)
                            u[e] = (float)q2[r][f][blk][e] > 0.f ? u[e] : u[e] * slope;
                        else
                            u[e] = u[e] >= 0.f ? u[e] : u[e] * slope;
                        if (fold) u[e] = u[e] * s1;
                        if (has_r2) {
                            u[e] = u[e] * s2 + (float)q2[r][f][blk][e];
                        } else {
                            if (scale2) u[e] *= s2;
                        }
                        if (!valid) u[e] = 0.f;
                    }
                    const auto yr = rsrc_n(ybase + (size_t)(2 * f + blk) * c.pstride, c.pstride);
                    bf16x8 tq;
#pragma unroll
                    for (int e = 0; e < 8; ++e) tq[e] = (__bf16)u[e];
                    if (!(c.abl & 4))
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tq), yr, pix * 32 + 16 * hh, 0, 16);
                }
            }
        }
    }
    publish_prev();
    // published after the next tile's first chunk (or before any wait that could need it)
    pb.pend = true;
    pb.t = t;
    pb.tseq = tseq;
    pb.v = c.gen * 1024u + (unsigned)(L + 1);
}

// 512 threads, one workgroup per CU (2 waves per SIMD: up to 256 VGPRs)
__global__ __launch_bounds__(lc::NT, 1) void trunk_lc_kernel(LcArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LcCtx c;
    c.state = a.state;
    c.acquire = a.acquire;
    c.gen = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const_geo& g = *(const_geo*)(uintptr_t)(a.state + a.rec_off - 16);
    const_rec* recs = (const_rec*)(uintptr_t)(a.state + a.rec_off);
    if (g.err != 0) {  // the prep kernel refused the layer table: give up loudly
        if (threadIdx.x == 0) {
            __hip_atomic_store(a.state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(a.state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    c.hp = g.hp;
    c.wp = g.wp;
    c.cs16 = g.cs16;
    c.pad = g.pad;
    c.h = g.h;
    c.w = g.w;
    c.nbx = g.nbx;
    c.nby = g.nby;
    c.ntiles = g.ntiles;
    c.pstride = (uint32_t)(c.hp * c.wp * 32);
    c.abl = lc_abl_load();
    // the compute waves walk a tile's chunks in pairs (alternating fragment sets): cin % 32 == 0
    bool even = true;
    for (int L = 0; L < a.nl; ++L) even = even && (rec_nch(recs[L]) % 2 == 0);
    if (!even) {
        if (threadIdx.x == 0 && blockIdx.x == 0) {
            __hip_atomic_store(a.state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(a.state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (threadIdx.x < 16) reinterpret_cast<unsigned*>(smem + lc::FLAG_OFF)[threadIdx.x] = 0u;
    __syncthreads();
    const int G = gridDim.x, b = blockIdx.x, wave = wave_id();
    if (b >= c.ntiles) return;
    if (wave >= lc::WMC) {
        lc_loader(c, recs, a.nl, G, b, wave - lc::WMC);
        return;
    }
    unsigned item = 0;
    int tseq = 0;
    LcPub pb;
    pb.pend = false;
    pb.t = pb.tseq = 0;
    pb.v = 0;
    for (int L = 0; L < a.nl; ++L) {
        const_rec& rec = recs[L];
        const int kind = rec_kind(rec);
        for (int t = b; t < c.ntiles; t += G, ++tseq) {
            if (kind == 0) lc_tile<1, false>(c, item, pb, tseq, rec, L, t, wave);
            else if (kind == 2) lc_tile<1, true>(c, item, pb, tseq, rec, L, t, wave);
            else lc_tile<2, false>(c, item, pb, tseq, rec, L, t, wave);
        }
    }
    lc_publish(c, pb);
}

// Grid: one workgroup per CU, every one resident (tiles wait on other workgroups' tiles).
int trunk_lc_launch(const isr_chain_desc* cd, hipStream_t s) {
    if (cd->ha % lc::TH || cd->wa % tk::TW || cd->nl < 1 || cd->nl > 1024) return -2;
    const long long ntiles = (long long)cd->n * (cd->wa / tk::TW) * (cd->ha / lc::TH);
    if (ntiles <= 0 || ntiles > (1 << 24)) return -2;
    static thread_local int cached_dev = -1, cached_per_cu = 0, cached_cus = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    const void* kern = (const void*)trunk_lc_kernel;
    if (dev != cached_dev) {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lc::LDS);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, lc::NT, lc::LDS) != hipSuccess) return -1;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return -1;
        cached_dev = dev;
        cached_per_cu = per_cu < 1 ? per_cu : 1;
        cached_cus = cus;
    }
    if (cached_per_cu < 1) return -4;
    const int grid = (int)(ntiles < cached_cus ? ntiles : cached_cus);
    const int rec_off = (int)trunk_rec_off((int)ntiles);
    if (trunk_prep_launch(cd, lc::TH, s) != 0) return -1;
    LcArgs a;
    a.state = cd->state;
    a.rec_off = rec_off;
    a.nl = cd->nl;
    a.acquire = cd->acquire;
    hipLaunchKernelGGL(trunk_lc_kernel, dim3(grid), dim3(lc::NT), lc::LDS, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#endif  // ISR_TUNING

}  // namespace isr
