// The RRDB trunk (utils/models.py:298-317 RRDB.forward over :245-271 RDB.forward, the
// `nn.Sequential(*RRDB)` of ResNet/EResNet :598 / :627) as ONE persistent launch — the round-4
// "deep ring" form (isr_conv_chain variant 4).
//
// Why a new main loop.  The round-3 pair form (trunk.hip, two 4-wave workgroups per CU, one
// 16-channel K-chunk in flight) spent per chunk and wave ~1,250 cycles waiting for its own
// LDS-DMA, ~700 in the barrier and ~2,800 issuing the step-0 fragment reads plus a block of 7-11
// LDS-DMA pieces, against 1,152 (growth) / 2,304 (final) cycles of its own MFMAs (profiles/
// r03_trunk_items_pair.jsonl): the chunk's fixed cost exceeded its matrix work, and two waves per
// SIMD can hide at most one such wave.  This form changes the structure, not the order of
// operations (outputs stay bit-identical to the per-conv launches):
//  * one 8-wave workgroup per CU on a 32 x 32 tile (4 output rows x 32 px per wave, as the pair
//    form): each chunk's weights are staged once per CU instead of twice, the halo is
//    (34 x 34) / (32 x 32) instead of (18 x 34) / (16 x 32) — 21-28 % fewer LDS-DMA bytes per FLOP;
//  * split rings: 3 halo slots (37 KB) and 2 weight slots (18 KB), so the halo of chunk i+3 is
//    issued while chunk i computes (~1.7 chunks of lead instead of < 1) — the LDS the pair form
//    spent on a second workgroup buys ring depth here;
//  * the chunk's barrier sits BEFORE its last MFMA step (dx = 2), after its last fragment read:
//    passing it frees the chunk's slots for refill and publishes the next chunk's slots, whose
//    step-0 fragments are then read inside the dx = 2 MFMAs — the matrix pipe no longer drains
//    across the barrier and the first fragment reads;
//  * no LDS-DMA block: each wave's pieces are spread over the MFMA stream (halo of chunk i+3 over
//    step 0 of chunk i+1; weights of chunk i+2, the bias and the dependency poll over step 2 of
//    chunk i), at fixed positions;
//  * the 3 x 3 tile-neighbourhood poll is itself an LDS-DMA (9 sc1 words into an LDS poll slot,
//    read by every wave after the next barrier): no wave drains its vector-memory queue to poll.
//    Only when the compute cursor reaches a chunk whose halo could not be staged (its producers
//    are not done) does a wave block — after publishing its own finished tile, so no wait cycle
//    can form.
// Hand-off per cdna_hip_programming.md Guideline 16 (R1), as trunk.hip: write-through (sc1)
// stores, every storing wave's vmcnt wait before a workgroup barrier, then a relaxed agent-scope
// progress store gen * 1024 + layers done; consumers poll with sc1 loads and read activations with
// sc1 LDS-DMA only after the poll matched.  Buffer resources carry the buffers' real extents, so
// an out-of-range offset reads zeros / drops the store instead of touching another allocation.
#include "trunk_common.h"

namespace isr {

// An A/B form (7.54 vs 6.36 ms per forward): compiled into the tuning library only.
#ifdef ISR_TUNING

namespace td {
constexpr int TH = 32, TW = 32, WM = 8, R = 4, NT = 64 * WM;
constexpr int HC = TW + 2, HQ = (TH + 2) * HC;  // 34 x 34 halo pixels
constexpr int HP = (HQ + 31) / 32;              // 37 halo pieces of 1 KB (the last one partial)
constexpr int HPW = (HP + WM - 1) / WM;         // halo pieces per wave (at most 5)
constexpr int WPF = 18, WPW = (WPF + WM - 1) / WM;  // weight pieces of a final conv chunk; per wave
constexpr int HSLOT = HP * 1024, WSLOT = WPF * 1024;
constexpr int NSH = 3, NSW = 2;                 // halo / weight ring depths
constexpr int W_OFF = NSH * HSLOT;
constexpr int BIAS_OFF = W_OFF + NSW * WSLOT;   // 4 bias slots of 256 B (by tile sequence)
constexpr int POLL_OFF = BIAS_OFF + 4 * 256;    // 2 poll slots of 64 words (by item parity)
constexpr int DUMMY_OFF = POLL_OFF + 2 * 256;   // 1 KB sink of inactive LDS-DMA pieces
constexpr int TBL_OFF = DUMMY_OFF + 1024;       // the workgroup's tile table (8 B per tile)
constexpr int MAX_TILES = 1024;                 // tiles per workgroup (the launcher refuses more)
constexpr int LDS = TBL_OFF + 8 * MAX_TILES;
static_assert(LDS <= 163840, "LDS budget");
static_assert(HQ / 34 == TH + 2 && tk::HC == HC, "halo image geometry shared with halo_piece_off");
}  // namespace td

#ifdef ISR_TUNING
__device__ int g_trunkd_knobs[4];
// event counters (tuning builds): [0] top slow paths, [1] their blocking waits, [2] mid-chunk slow
// paths, [3] their blocking waits, [4] polls issued, [5] polls that found the neighbourhood done
__device__ unsigned long long g_trunkd_stats[8];
__device__ __forceinline__ int trunkd_abl() { return __builtin_amdgcn_readfirstlane(g_trunkd_knobs[0]); }
__device__ __forceinline__ void trunkd_count(int k) {
    if (threadIdx.x == 0) atomicAdd(&g_trunkd_stats[k], 1ull);
}
// per-chunk cycle stamps (s_memtime) of layers 77 (growth2) and 79 (final), each workgroup's first
// tile, lane 0 of waves 0 and 4: [grid][2][16 chunks][2][8]: [0] chunk top, [1] step-0 fragments
// requested, [2] steps 0-1 issued, [3] own DMA waited, [4] barrier passed, [5] decisions done,
// [6] step 2 issued
__device__ unsigned long long* g_trunkd_stamps;
__device__ __forceinline__ void trunkd_stamp(int L, int k, int ch, int slot) {
    unsigned long long* p = g_trunkd_stamps;
    const int w = wave_id();
    if (p != nullptr && k == 0 && (threadIdx.x & 63) == 0 && (w == 0 || w == 4) && (L == 77 || L == 79) && ch < 16) {
        const unsigned long long v = __builtin_amdgcn_s_memtime();
        p[((((size_t)blockIdx.x * 2 + (L == 79)) * 16 + ch) * 2 + (w != 0)) * 8 + slot] = v;
    }
}
#else
__device__ __forceinline__ int trunkd_abl() { return 0; }
__device__ __forceinline__ void trunkd_count(int) {}
__device__ __forceinline__ void trunkd_stamp(int, int, int, int) {}
#endif

// Per-workgroup tile table in LDS (written once at kernel start; the workgroup's tiles are
// t = b + k G for k < my_tiles, the same list on every layer): [k] = {halo origin byte offset of
// the tile at plane 0 of its image: pixel (y0 - 1, x0 - 1); img | by << 10 | bx << 21}.  Keeps the
// tile -> (img, by, bx) divisions out of the MFMA stream.
struct DCtx {
    unsigned* state;
    const_rec* recs;
    unsigned gen;
    int nl, G, b, my_tiles;
    uint32_t nbxy;               // tiles per row | per column << 16
    uint32_t pstride, abytes;    // bytes per 16-channel plane; bytes of one activation buffer
    uint32_t hoff[td::HPW];      // per-lane halo piece offsets (chunk-invariant)
    int abl;
};

__device__ __forceinline__ const_geo& geo_of(const DCtx& c) {
    return *(const_geo*)((const __attribute__((address_space(4))) char*)c.recs - 64);
}

// A position in the workgroup's item stream, packed: L << 21 | k << 8 | ch (item = K-chunk ch of
// the workgroup's tile k of layer L).  Wave-uniform.
__device__ __forceinline__ int cL(uint32_t p) { return (int)(p >> 21); }
__device__ __forceinline__ int cK(uint32_t p) { return (int)((p >> 8) & 8191); }
__device__ __forceinline__ int cCH(uint32_t p) { return (int)(p & 255); }
// A cursor may stand past the stream's last layer (it stops there); the branch-free staging code
// still reads its layer's record, so record reads clamp to the last layer (nl may be 1024, the
// records' capacity).
__device__ __forceinline__ const_rec& rec_at(const DCtx& c, int L) { return c.recs[L < c.nl ? L : c.nl - 1]; }

// A cursor's layer in one word (kept beside the cursor, re-read from the record only when the
// cursor changes layer — record loads on the barrier's critical path cost ~1,000 cycles per chunk):
// nch | first_new << 8 | xp << 16 | wpc << 24.
__device__ __forceinline__ uint32_t lay_info(const DCtx& c, int L) {
    const_rec& r = rec_at(c, L);
    return (uint32_t)rec_nch(r) | (uint32_t)rec_first_new(r) << 8 | (uint32_t)rec_xp(r) << 16 |
           (uint32_t)(rec_kind(r) == 0 ? tk::WPG : tk::WPF) << 24;
}
__device__ __forceinline__ int inf_nch(uint32_t f) { return (int)(f & 255); }
__device__ __forceinline__ int inf_fnew(uint32_t f) { return (int)((f >> 8) & 255); }
__device__ __forceinline__ int inf_xp(uint32_t f) { return (int)((f >> 16) & 255); }
__device__ __forceinline__ int inf_wpc(uint32_t f) { return (int)(f >> 24); }

// advance cursor p (layer info f) by one item; a layer change re-reads f
__device__ __forceinline__ void cur_adv(const DCtx& c, uint32_t& p, uint32_t& f) {
    const int L = cL(p), k = cK(p);
    if (cCH(p) + 1 < inf_nch(f)) {
        ++p;
    } else if (k + 1 < c.my_tiles) {
        p = (uint32_t)L << 21 | (uint32_t)(k + 1) << 8;
    } else {
        p = (uint32_t)(L + 1) << 21;
        f = lay_info(c, L + 1);
    }
}

// bias slot of the cursor's tile: the workgroup's tile sequence number & 3
__device__ __forceinline__ int cur_bslot(const DCtx& c, uint32_t p) { return (cL(p) * c.my_tiles + cK(p)) & 3; }

// The tile's halo needs its neighbourhood done with layer L-1 before this chunk is staged: the
// chunks from the first one layer L-1 wrote; every chunk of a layer that reads nothing its
// predecessor wrote (so that every tile of layer >= 1 confirms its neighbourhood before its
// stores land, and the next layer's older chunks are final when its cursor gets there).
__device__ __forceinline__ bool cur_needs_dep(uint32_t p, uint32_t f) {
    if (cL(p) == 0) return false;
    const int fnew = inf_fnew(f);
    return fnew != tk::NEED_NONE && (cCH(p) >= fnew || fnew >= inf_nch(f));
}

__device__ __forceinline__ uint32_t tbl_hbase(int k) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    return *reinterpret_cast<const uint32_t*>(smem + td::TBL_OFF + k * 8);
}
__device__ __forceinline__ uint32_t tbl_pos(int k) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    return *reinterpret_cast<const uint32_t*>(smem + td::TBL_OFF + k * 8 + 4);
}

// Neighbour polled by this lane (lanes 0..8: the 3 x 3 neighbourhood of the tile at `pos`), or -1.
__device__ __forceinline__ int nb_of_pos(const DCtx& c, uint32_t pos) {
    const int lane = threadIdx.x & 63;
    const int img = (int)(pos & 1023), by = (int)((pos >> 10) & 2047), bx = (int)(pos >> 21);
    const int yy = by + lane / 3 - 1, xx = bx + lane % 3 - 1;
    const int nbx = (int)(c.nbxy & 0xffff), nby = (int)(c.nbxy >> 16);
    return (lane < 9 && yy >= 0 && yy < nby && xx >= 0 && xx < nbx) ? (img * nby + yy) * nbx + xx : -1;
}

// Per wave, carried through the whole stream (all wave-uniform).
struct DStream {
    int i;                 // item being computed
    int wi, hi;            // next item whose weights / halo are not staged yet
    uint32_t wcur, hcur;   // their positions
    uint32_t winf, hinf;   // their layers' info words (lay_info)
    uint32_t hso;          // halo source offset of item hi (set with F_GO_H)
    uint32_t fl;           // flags (F_*), packed: wave-uniform bools would take an SGPR pair each
    uint32_t issued;       // vector-memory instructions issued by this wave
    uint32_t mk0, mk1, mk2, mk3;  // mark of item j (at j & 3): `issued` after its last piece
    uint32_t poll_mark;    // `issued` after the outstanding poll (F_POLL)
    uint32_t poll_tile;    // its tile (the cursor's L, k: hcur >> 8 when it was issued)
    int pend;              // the finished tile whose progress word waits for its stores:
                           // t << 11 | (L + 1), or -1
    uint32_t pend_mark;
};

// DStream::fl bits.  GO_*: decided at a barrier, carried out at fixed positions of the next MFMA
// steps (weights / halo of the next unstaged items, a neighbourhood poll); HDEP: the halo
// cursor's tile has its neighbourhood confirmed; READY: the next item's slots are staged, landed
// and visible; FRAGS: its step-0 fragments are already in registers (set P^1).
enum : uint32_t { F_GO_W = 1, F_GO_H = 2, F_GO_POLL = 4, F_HDEP = 8, F_READY = 16, F_FRAGS = 32, F_POLL = 64,
                  F_POLLP = 128 };  // POLL: a poll is outstanding, in poll slot POLLP
__device__ __forceinline__ bool has(const DStream& s, uint32_t f) { return (s.fl & f) != 0; }
__device__ __forceinline__ void setf(DStream& s, uint32_t f, bool v) { s.fl = v ? (s.fl | f) : (s.fl & ~f); }

__device__ __forceinline__ void set_mark(DStream& s, int j, uint32_t v) {
    const int k = j & 3;
    s.mk0 = k == 0 ? v : s.mk0;
    s.mk1 = k == 1 ? v : s.mk1;
    s.mk2 = k == 2 ? v : s.mk2;
    s.mk3 = k == 3 ? v : s.mk3;
}

__device__ __forceinline__ uint32_t get_mark(const DStream& s, int j) {
    const int k = j & 3;
    return k == 0 ? s.mk0 : (k == 1 ? s.mk1 : (k == 2 ? s.mk2 : s.mk3));
}

// halo source offset of the cursor's item, from the tile table's base `hb`
__device__ __forceinline__ uint32_t halo_src(const DCtx& c, uint32_t p, uint32_t f, uint32_t hb) {
    return hb + (uint32_t)(inf_xp(f) + cCH(p)) * c.pstride;
}

// ---- staging pieces: one LDS-DMA instruction each when active (wave-uniform branch) ----
template <int K>
__device__ __forceinline__ void stage_h_piece(const DCtx& c, DStream& s) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int j = wave_id() + td::WM * K;
    if (!has(s, F_GO_H) || j >= td::HP || (c.abl & 1)) return;
    const_rec& r = rec_at(c, cL(s.hcur));
    char* dst = smem + (s.hi % td::NSH) * td::HSLOT + j * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n((const void*)(uintptr_t)r.x, c.abytes), ISR_LDS_PTR(dst), 16,
                                             c.hoff[K], s.hso, 0, 16);
    ++s.issued;
}

__device__ __forceinline__ void finish_h(const DCtx& c, DStream& s) {
    if (!has(s, F_GO_H)) return;
    set_mark(s, s.hi, s.issued);
    ++s.hi;
    const uint32_t old = s.hcur;
    cur_adv(c, s.hcur, s.hinf);
    if ((s.hcur >> 8) != (old >> 8)) setf(s, F_HDEP, false);  // a new tile: not confirmed yet
    setf(s, F_GO_H, false);
}

template <int K>
__device__ __forceinline__ void stage_w_piece(const DCtx& c, DStream& s) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, j = wave_id() + td::WM * K;
    const int L = cL(s.wcur), wpc = inf_wpc(s.winf);
    if (!has(s, F_GO_W) || j >= wpc || (c.abl & 8)) return;
    const_rec& r = rec_at(c, L);
    const uint32_t wbytes = (uint32_t)(inf_nch(s.winf) * wpc * 1024);
    char* dst = smem + td::W_OFF + (s.wi & 1) * td::WSLOT + j * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n((const void*)(uintptr_t)r.w, wbytes), ISR_LDS_PTR(dst), 16,
                                             lane * 16, (uint32_t)(cCH(s.wcur) * wpc + j) * 1024, 0, 0);
    ++s.issued;
}

// the bias of a tile's first chunk (wave 0: 4 B per lane; lanes beyond cout read zeros)
__device__ __forceinline__ void stage_bias(const DCtx& c, DStream& s) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (!has(s, F_GO_W) || cCH(s.wcur) != 0 || wave_id() != 0) return;
    const int L = cL(s.wcur);
    const int lane = threadIdx.x & 63, cout = inf_wpc(s.winf) == tk::WPG ? 32 : 64;
    const_rec& r = rec_at(c, L);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n((const void*)(uintptr_t)r.b, (uint32_t)cout * 4),
                                             ISR_LDS_PTR(smem + td::BIAS_OFF + cur_bslot(c, s.wcur) * 256), 4,
                                             lane * 4, 0, 0, 0);
    ++s.issued;
}

__device__ __forceinline__ void finish_w(const DCtx& c, DStream& s) {
    if (!has(s, F_GO_W)) return;
    set_mark(s, s.wi, s.issued);
    ++s.wi;
    cur_adv(c, s.wcur, s.winf);
    setf(s, F_GO_W, false);
}

// the neighbourhood poll of the halo cursor's tile (this lane's neighbour nb, from d_barrier):
// 9 progress words (sc1) into poll slot (item & 1) by wave 0; read by every wave after the
// barrier that follows its vmcnt wait
__device__ __forceinline__ void stage_poll(const DCtx& c, DStream& s, int nb) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (!has(s, F_GO_POLL)) return;
    if (wave_id() == 0) {
        if (nb >= 0)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n(c.state, (uint32_t)(4 + geo_of(c).ntiles) * 4),
                                                     ISR_LDS_PTR(smem + td::POLL_OFF + (s.i & 1) * 256), 4,
                                                     (uint32_t)(4 + nb) * 4, 0, 0, 16);
        ++s.issued;
    }
    setf(s, F_POLL, true);
    setf(s, F_POLLP, (s.i & 1) != 0);
    s.poll_mark = s.issued;
    s.poll_tile = s.hcur >> 8;
    setf(s, F_GO_POLL, false);
}

// Every piece of the halo cursor's item at once (slow path and prologue).
__device__ __forceinline__ void stage_h_block(const DCtx& c, DStream& s) {
    setf(s, F_GO_H, true);
    s.hso = halo_src(c, s.hcur, s.hinf, __builtin_amdgcn_readfirstlane(tbl_hbase(cK(s.hcur))));
    stage_h_piece<0>(c, s);
    stage_h_piece<1>(c, s);
    stage_h_piece<2>(c, s);
    stage_h_piece<3>(c, s);
    stage_h_piece<4>(c, s);
    static_assert(td::HPW == 5, "halo pieces per wave");
    finish_h(c, s);
}

__device__ __forceinline__ void stage_w_block(const DCtx& c, DStream& s) {
    setf(s, F_GO_W, true);
    stage_w_piece<0>(c, s);
    stage_w_piece<1>(c, s);
    stage_w_piece<2>(c, s);
    stage_bias(c, s);
    static_assert(td::WPW == 3, "weight pieces per wave");
    finish_w(c, s);
}

// The pending tile's progress word (lane 0 of wave 0, after a barrier every storing wave passed
// behind its own vmcnt wait).
__device__ __forceinline__ void d_publish(const DCtx& c, DStream& s) {
    if (threadIdx.x == 0)
        __hip_atomic_store(c.state + 4 + (s.pend >> 11), c.gen * 1024u + (unsigned)(s.pend & 2047), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    s.pend = -1;
}

// Publish the pending tile now: every wave drains its vector memory, workgroup barrier, flag.
// Before any blocking wait (no workgroup may spin on a word this one holds back).
__device__ __forceinline__ void d_force_publish(const DCtx& c, DStream& s) {
    if (s.pend < 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    d_publish(c, s);
}

// Slow path at the top of item i: its slots were not staged or not published by the previous
// barrier.  Stage what is missing (blocking on the neighbourhood if needed, after publishing our
// own pending tile), then wait for this wave's pieces and make every wave's visible.
__device__ __forceinline__ void d_slow_path(const DCtx& c, DStream& s) {
    const int i = s.i;
    trunkd_count(0);
    if (s.wi <= i) stage_w_block(c, s);  // (weights never wait on anything: normally staged)
    if (s.hi <= i) {
        setf(s, F_POLL, false);  // an outstanding poll would be read for the cursor's tile after it moved
        if (cur_needs_dep(s.hcur, s.hinf) && !has(s, F_HDEP)) {
            trunkd_count(1);
            d_force_publish(c, s);
            if (!(c.abl & 16)) {
                const int nb = nb_of_pos(c, tbl_pos(cK(s.hcur)));
                dep_wait(c.state, nb, c.gen * 1024u + (unsigned)cL(s.hcur), c.gen);
            }
            setf(s, F_HDEP, true);
        }
        stage_h_block(c, s);
        // refill the ring while the dependency is known to hold (same tile)
        while (s.hi <= i + 2 && cL(s.hcur) < c.nl && (!cur_needs_dep(s.hcur, s.hinf) || has(s, F_HDEP)))
            stage_h_block(c, s);
    }
    if (s.wi <= i + 1 && cL(s.wcur) < c.nl) stage_w_block(c, s);
    const uint32_t tgt = get_mark(s, i);
    wait_vm(s.issued - tgt);
    raw_barrier();
    if (s.pend >= 0 && (int)(tgt - s.pend_mark) >= 0) d_publish(c, s);
}

// The chunk barrier of item i (before its dx = 2 step): every wave's reads of item i's slots are
// done (lgkmcnt(0) in raw_barrier), its own pieces of item i+1 (and the pending tile's stores,
// and an outstanding poll) have landed.  After it: publish, read the poll, and, when item i+1
// continues this tile (MORE: its step-0 fragments are read right behind this barrier) but was
// not staged, stage it now — blocking on the neighbourhood if needed; safe mid-tile: the wait is
// for layer L-1 of the neighbours, never for this workgroup's unfinished tile, and its previous
// tile was just published — then a second barrier.  Last, decide the next period's staging
// (weights of i+2, halo of up to i+3).  Returns this lane's neighbour of the halo cursor's tile
// (for a poll to issue).
template <bool MORE>
__device__ __forceinline__ int d_barrier(const DCtx& c, DStream& s, int sL, int sk, int sch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int i = s.i;
    const bool next_staged = s.wi > i + 1 && s.hi > i + 1;  // (the cursors stop at the stream's end)
    uint32_t tgt = s.issued;  // sentinel: nothing to wait for
    bool any = false;
    auto want = [&](uint32_t m) {
        if (!any || (int)(m - tgt) > 0) tgt = m;
        any = true;
    };
    if (next_staged) want(get_mark(s, i + 1));
    if (s.pend >= 0) want(s.pend_mark);
    if (has(s, F_POLL)) want(s.poll_mark);
    if (any) wait_vm(s.issued - tgt);
    trunkd_stamp(sL, sk, sch, 3);
    // the halo cursor's tile: read before the barrier (its lgkmcnt(0) covers the reads)
    int hk = cK(s.hcur);
    uint32_t hb = tbl_hbase(hk), hpos = tbl_pos(hk);
    raw_barrier();
    trunkd_stamp(sL, sk, sch, 4);
    setf(s, F_READY, next_staged);
    if (s.pend >= 0) d_publish(c, s);
    int nb = nb_of_pos(c, hpos);
    // the poll issued at an earlier barrier has landed in its slot: the neighbourhood's verdict
    if (has(s, F_POLL) && s.poll_tile == (s.hcur >> 8)) {  // (a poll of a tile the cursor has left is void)
        const int lane = threadIdx.x & 63;
        const unsigned v = *reinterpret_cast<const volatile unsigned*>(smem + td::POLL_OFF +
                                                                       (has(s, F_POLLP) ? 256 : 0) + lane * 4);
        const unsigned need = c.gen * 1024u + (unsigned)cL(s.hcur);  // done with layer L - 1
        if (__all(nb < 0 || (int)(v - need) >= 0)) {
            setf(s, F_HDEP, true);
            trunkd_count(5);
        }
    }
    setf(s, F_POLL, false);
    if (MORE && !next_staged) {
        trunkd_count(2);
        if (s.wi <= i + 1) stage_w_block(c, s);
        if (s.hi <= i + 1) {
            if (cur_needs_dep(s.hcur, s.hinf) && !has(s, F_HDEP)) {
                trunkd_count(3);
                if (!(c.abl & 16)) dep_wait(c.state, nb, c.gen * 1024u + (unsigned)cL(s.hcur), c.gen);
                setf(s, F_HDEP, true);
            }
            stage_h_block(c, s);
        }
        wait_vm(s.issued - get_mark(s, i + 1));
        raw_barrier();
        setf(s, F_READY, true);
        hk = cK(s.hcur);
        hb = __builtin_amdgcn_readfirstlane(tbl_hbase(hk));
        nb = nb_of_pos(c, tbl_pos(hk));
    }
    // weights of the next unstaged item (normally i+2; its slot held item i, free now)
    setf(s, F_GO_W, s.wi <= i + 2 && cL(s.wcur) < c.nl);
    // halo of the next unstaged item up to i+3 (its slot held item hi-3 <= i)
    setf(s, F_GO_H, false);
    if (s.hi <= i + 3 && cL(s.hcur) < c.nl) {
        if (!cur_needs_dep(s.hcur, s.hinf) || has(s, F_HDEP) || (c.abl & 16)) {
            setf(s, F_GO_H, true);
            s.hso = halo_src(c, s.hcur, s.hinf, __builtin_amdgcn_readfirstlane(hb));
        }
    }
    // poll the cursor tile's neighbourhood from the tile's first chunk on (not only once the
    // cursor stands at a chunk that needs it): the verdict is one barrier old when it is read
    if (cL(s.hcur) > 0 && cL(s.hcur) < c.nl && !has(s, F_HDEP) && !(c.abl & 16) &&
        inf_fnew(s.hinf) != tk::NEED_NONE) {
        setf(s, F_GO_POLL, true);
        trunkd_count(4);
    }
    return nb;
}

template <int V> struct PIC { static constexpr int value = V; };

// One tile of one layer: NF = 1 (growth, 32 couts) or 2 (final, 64 couts).
template <int NF>
__device__ __forceinline__ void d_run_tile(const DCtx& c, DStream& s, const_rec& rec, const int L, const int k) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = td::R, CT = 32 * NF, TN = 3;
    const int wave = wave_id(), lane = threadIdx.x & 63, l31 = lane & 31, hh = lane >> 5;
    const bool grp_b = wave >= 4;
    const int t = c.b + k * c.G, nch = rec_nch(rec);
    const uint32_t pos = __builtin_amdgcn_readfirstlane(tbl_pos(k));
    const int img = (int)(pos & 1023), by = (int)((pos >> 10) & 2047), bx = (int)(pos >> 21);
    const int x0 = bx * td::TW, y0 = by * td::TH;
    const bool fold = NF == 2 && rec_fold(rec);
    const bool has_r2 = NF == 2 && rec.r2 != 0;
    const uint32_t idv = rec_idv(rec);
    const int bslot = (L * c.my_tiles + k) & 3;

    // per-lane LDS read addresses relative to a slot: weights A[n][k] (n = cout), halo rows
    const uint32_t a_w = (uint32_t)((2 * l31 + (hh ^ ((l31 >> 3) & 1))) * 16);
    uint32_t a_h[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
        a_h[dx] = (uint32_t)((wave * R * td::HC + l31 + dx) * 32 + 16 * (hh ^ (((l31 + dx) >> 3) & 1)));

    f32x16 acc[R][NF];
    // fragment register sets (local to the tile: nothing is prefetched across a tile boundary, so
    // they are dead in the epilogue)
    bf16x8 fb[2][TN][NF], fa[2][R + 2];

    // fragment reads of step dx from the slots of item `it` into register set `set`
    auto read_one = [&](int it, int dx, int idx, int set) {
        const char* hs = smem + (it % td::NSH) * td::HSLOT;
        const char* ws = smem + td::W_OFF + (it & 1) * td::WSLOT;
        if (idx < TN * NF) {
            const int dyi = idx / NF, f = idx % NF;
            fb[set][dyi][f] = lds_read16(ws + a_w + ((dyi * 3 + dx) * CT * 2 + f * 64) * 16);
        } else {
            const int ia = idx - TN * NF;
            fa[set][ia] = lds_read16(hs + a_h[dx] + ia * td::HC * 32);
        }
    };
    auto read_step0 = [&](int it, int set) {
#pragma unroll
        for (int f = 0; f < NF; ++f) read_one(it, 0, f, set);
#pragma unroll
        for (int ia = 0; ia < R; ++ia) read_one(it, 0, TN * NF + ia, set);
#pragma unroll
        for (int f = 0; f < NF; ++f) read_one(it, 0, NF + f, set);
        read_one(it, 0, TN * NF + R, set);
#pragma unroll
        for (int f = 0; f < NF; ++f) read_one(it, 0, 2 * NF + f, set);
        read_one(it, 0, TN * NF + R + 1, set);
    };

    // one K-chunk.  P: the register set of its step 0 (chunks alternate; nch is even, so a tile's
    // chunk ch runs with P = ch & 1).  Staging positions: halo pieces at step-0 MFMA rows
    // (dyi, r) = (0, 0..3), (1, 0); poll, weight pieces and bias at step-2 rows (0, 0..3), (1, 0).
    // The residual fold of chunks 0..3 (couts 16 ch .. + 16: fragment ch >> 1, half P) adds its
    // 4 MFMAs after step 1's dy = 1 rows, i.e. between each accumulator's dy = 1 and dy = 2
    // contributions of dx = 1 — the same point of the same order as conv3x3.hip.
    auto chunk = [&](const int ch, auto p_tag, auto more_tag, auto fold_tag, auto first_tag) {
        constexpr int P = decltype(p_tag)::value;
        constexpr bool MORE = decltype(more_tag)::value != 0;    // the next item continues this tile
        constexpr int FF = decltype(fold_tag)::value;            // fold target fragment (chunks 0..3), or -1
        constexpr bool FIRST = decltype(first_tag)::value != 0;  // the tile's chunk 0: nothing prefetched
        const int it = s.i;
        trunkd_stamp(L, k, ch, 0);
        if constexpr (FIRST) {
            if (!has(s, F_READY)) d_slow_path(c, s);
            read_step0(it, P);
        }
        trunkd_stamp(L, k, ch, 1);
        setf(s, F_READY, false);
        int pnb = -1;
        if (ch == 0) {
            // bias → accumulators (register g of lane l: cout (g&3) + 8(g>>2) + 4hh of fragment f)
            const float* bs = reinterpret_cast<const float*>(smem + td::BIAS_OFF + bslot * 256);
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
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int stp = 0; stp < 3; ++stp) {
            const int cur = (P + stp) & 1;
            if (stp == 2) {
                __builtin_amdgcn_s_setprio(0);
                trunkd_stamp(L, k, ch, 2);
                pnb = d_barrier<MORE>(c, s, L, k, ch);
                trunkd_stamp(L, k, ch, 5);
                __builtin_amdgcn_s_setprio(1);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int dyi = 0; dyi < TN; ++dyi) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
#pragma unroll
                    for (int f = 0; f < NF; ++f) acc[r][f] = mfma32(fb[cur][dyi][f], fa[cur][r + dyi], acc[r][f]);
                    // input row ia = r + dyi is last used here when dyi == min(2, ia)
                    if (dyi == 2 || r == 0) {
                        if (stp < 2) read_one(it, stp + 1, TN * NF + r + dyi, cur ^ 1);
                        else if (MORE) read_one(it + 1, 0, TN * NF + r + dyi, cur ^ 1);
                    }
                    // spread staging
                    // waves 0-3 and their SIMD partners 4-7 issue at positions 6 rows apart, so
                    // the two waves of a SIMD never stall on LDS-DMA issue at the same MFMA
                    const int q = dyi * R + r - (grp_b ? 6 : 0);
                    if (stp == 0) {
                        if (q == 0) stage_h_piece<0>(c, s);
                        if (q == 1) stage_h_piece<1>(c, s);
                        if (q == 2) stage_h_piece<2>(c, s);
                        if (q == 3) stage_h_piece<3>(c, s);
                        if (q == 4) {
                            stage_h_piece<4>(c, s);
                            finish_h(c, s);
                        }
                    } else if (stp == 2) {
                        if (q == 0) stage_poll(c, s, pnb);
                        if (q == 1) stage_w_piece<0>(c, s);
                        if (q == 2) stage_w_piece<1>(c, s);
                        if (q == 3) stage_w_piece<2>(c, s);
                        if (q == 4) {
                            stage_bias(c, s);
                            finish_w(c, s);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if constexpr (NF == 2 && FF >= 0) {
                    if (stp == 1 && dyi == 1) {
                        // residual fold: + x/s1 on the centre pixels (dx = 1, dy = 1) of each row
                        // (compile-time target: a run-time choice made hipcc MFMA into temporaries)
                        const bf16x8 a = fold_a_bits(idv, P);
#pragma unroll
                        for (int r = 0; r < R; ++r) acc[r][FF] = mfma32(a, fa[cur][r + 1], acc[r][FF]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if (stp < 2) {
#pragma unroll
                    for (int f = 0; f < NF; ++f) read_one(it, stp + 1, dyi * NF + f, cur ^ 1);
                } else if (MORE) {
#pragma unroll
                    for (int f = 0; f < NF; ++f) read_one(it + 1, 0, dyi * NF + f, cur ^ 1);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        trunkd_stamp(L, k, ch, 6);
        ++s.i;
    };

    // chunk sequence: chunk 0 reads its step-0 fragments at the top (nothing is prefetched across
    // tiles), every later chunk gets them from the previous chunk's dx = 2 step; the register set
    // alternates (P = ch & 1, nch even).  A final conv (NF = 2) always folds (variant 4 needs it):
    // chunks 0..3 carry the residual fold.
    using T0 = PIC<0>;
    using T1 = PIC<1>;
    using TN1 = PIC<-1>;
    if constexpr (NF == 2) {
        chunk(0, T0{}, T1{}, T0{}, T1{});
        chunk(1, T1{}, T1{}, T0{}, T0{});
        chunk(2, T0{}, T1{}, T1{}, T0{});
        chunk(3, T1{}, T1{}, T1{}, T0{});
#pragma nounroll
        for (int ch = 4; ch < nch - 2; ch += 2) {
            chunk(ch, T0{}, T1{}, TN1{}, T0{});
            chunk(ch + 1, T1{}, T1{}, TN1{}, T0{});
        }
        chunk(nch - 2, T0{}, T1{}, TN1{}, T0{});
        chunk(nch - 1, T1{}, T0{}, TN1{}, T0{});
    } else {
        chunk(0, T0{}, T1{}, TN1{}, T1{});
#pragma nounroll
        for (int ch = 1; ch < nch - 1; ch += 2) {
            chunk(ch, T1{}, T1{}, TN1{}, T0{});
            chunk(ch + 1, T0{}, T1{}, TN1{}, T0{});
        }
        chunk(nch - 1, T1{}, T0{}, TN1{}, T0{});
    }
    (void)fold;

    // ---- epilogue: straight from the accumulators, write-through (sc1) stores ----
    {
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const int xx = x0 + l31;
        const auto yr = rsrc_n((const void*)(uintptr_t)rec.y, c.abytes);
        const float slope = rec.slope, s1 = rec.s1, s2 = rec.s2;
        const bool scale2 = s2 != 1.f;
        const_geo& g = geo_of(c);
        const int cs16 = g.cs16, hgt = g.h, wid = g.w, wp = g.wp, pad = g.pad;
        const uint32_t plane_px = c.pstride / 32;
        const uint32_t ypl = (uint32_t)(img * cs16 + rec_yp(rec)) * plane_px;
        bf16x8 q2[R][NF][2];
        const uint32_t r2pl = (uint32_t)(img * cs16 + rec_r2p(rec)) * plane_px;
        const auto rr = rsrc_n((const void*)(uintptr_t)rec.r2, c.abytes);
        auto load_r2 = [&](int r) {
            const uint32_t pix = (uint32_t)((y0 + wave * R + r + pad) * wp + xx + pad);
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const int co = f * 32 + 16 * blk + 8 * hh;
                    q2[r][f][blk] = __builtin_bit_cast(
                        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                    rr, (r2pl + (uint32_t)(co >> 4) * plane_px + pix) * 32 + 16 * hh, 0, 16));
                }
            s.issued += NF * 2;
        };
        if (has_r2) load_r2(0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (has_r2 && r + 1 < R) load_r2(r + 1);
            const int yy = y0 + wave * R + r;
            const bool valid = yy < hgt && xx < wid;
            const uint32_t pix = (uint32_t)((yy + pad) * wp + xx + pad);
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
                        u[e] = u[e] >= 0.f ? u[e] : u[e] * slope;
                        if (fold) u[e] = u[e] * s1;
                        if (has_r2) {
                            u[e] = u[e] * s2 + (float)q2[r][f][blk][e];
                        } else {
                            if (scale2) u[e] *= s2;
                        }
                        if (!valid) u[e] = 0.f;
                    }
                    const int co = f * 32 + 16 * blk + 8 * hh;
                    const uint32_t off = (ypl + (uint32_t)(co >> 4) * plane_px + pix) * 32 + 16 * hh;
                    bf16x8 tq;
#pragma unroll
                    for (int e = 0; e < 8; ++e) tq[e] = (__bf16)u[e];
                    if (!(c.abl & 4)) {
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tq), yr, off, 0, 16);
                        ++s.issued;
                    }
                }
            }
        }
    }
    s.pend = t << 11 | (L + 1);
    s.pend_mark = s.issued;
}

__global__ __launch_bounds__(td::NT, 2) void trunk_deep_kernel(unsigned* state, int rec_off, int nl) {
    DCtx c;
    c.state = state;
    c.gen = __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const_geo& g = *(const_geo*)(uintptr_t)(state + rec_off - 16);
    c.recs = (const_rec*)(uintptr_t)(state + rec_off);
    if (g.err != 0) {  // the prep kernel refused the layer table: give up loudly (once per launch)
        if (threadIdx.x == 0 && blockIdx.x == 0) {
            __hip_atomic_store(state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // this form pairs chunks (register sets alternate) and peels a final conv's 4 fold chunks
    // ahead of at least one more pair: every layer needs an even chunk count; a final conv the
    // residual fold and at least 6 chunks
    bool shape_ok = true;
    for (int L = 0; L < nl; ++L) {
        const int n = rec_nch(c.recs[L]);
        shape_ok = shape_ok && (n % 2 == 0) && n >= 2 && rec_kind(c.recs[L]) != 2 &&
                   (rec_kind(c.recs[L]) == 0 || (rec_fold(c.recs[L]) && n >= 6));  // no masked (kind 2) layers
    }
    // this A/B form addresses a whole activation buffer with 32-bit offsets: < 2 GiB only
    if ((size_t)g.n * g.cs16 * g.hp * g.wp * 32 >= 0x7fffffffull) shape_ok = false;
    if (!shape_ok) {
        if (threadIdx.x == 0 && blockIdx.x == 0) {
            __hip_atomic_store(state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    c.nl = nl;
    c.G = gridDim.x;
    c.b = blockIdx.x;
    const int ntiles = g.ntiles;
    c.my_tiles = c.b < ntiles ? (ntiles - 1 - c.b) / c.G + 1 : 0;
    c.nbxy = (uint32_t)g.nbx | (uint32_t)g.nby << 16;
    c.pstride = (uint32_t)(g.hp * g.wp * 32);
    c.abytes = (uint32_t)((size_t)g.n * g.cs16 * c.pstride);  // < 2 GiB (prep err bit 64)
    c.abl = trunkd_abl();
    {
        const int wave = wave_id(), lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < td::HPW; ++k) c.hoff[k] = halo_piece_off<td::HQ>(wave + td::WM * k, lane, g.wp);
    }
    // the tile table (launcher: my_tiles <= MAX_TILES)
    {
        extern __shared__ __attribute__((aligned(16))) char smem[];
        for (int k = threadIdx.x; k < c.my_tiles; k += td::NT) {
            const int t = c.b + k * c.G;
            const int bx = t % g.nbx, tmp = t / g.nbx, by = tmp % g.nby, img = tmp / g.nby;
            uint32_t* e = reinterpret_cast<uint32_t*>(smem + td::TBL_OFF + k * 8);
            e[0] = (uint32_t)img * (uint32_t)g.cs16 * c.pstride +
                   (uint32_t)(((by * td::TH - 1 + g.pad) * g.wp + (bx * td::TW - 1 + g.pad)) * 32);
            e[1] = (uint32_t)img | (uint32_t)by << 10 | (uint32_t)bx << 21;
        }
        __syncthreads();
    }
    DStream s;
    s.i = 0;
    s.issued = 0;
    s.mk0 = s.mk1 = s.mk2 = s.mk3 = 0;
    s.fl = 0;
    s.hso = 0;
    s.poll_mark = 0;
    s.poll_tile = 0;
    s.pend = -1;
    s.pend_mark = 0;
    s.wcur = s.hcur = 0;
    s.winf = s.hinf = lay_info(c, 0);
    s.wi = s.hi = 0;
    if (c.my_tiles > 0) {
        // prologue: weights of items 0, 1 and the halo of items 0..2 (layer 0 reads the trunk
        // input only: no dependency), then the first item's slow path makes them visible
        stage_w_block(c, s);
        stage_w_block(c, s);  // (every stream has >= 2 items: nch >= 2)
        stage_h_block(c, s);
        while (s.hi < 3 && cL(s.hcur) < c.nl && !cur_needs_dep(s.hcur, s.hinf)) stage_h_block(c, s);
        for (int L = 0; L < nl; ++L) {
            const_rec& rec = c.recs[L];
            const bool growth = rec_kind(rec) == 0;
            for (int k = 0; k < c.my_tiles; ++k) {
                if (growth) d_run_tile<1>(c, s, rec, L, k);
                else d_run_tile<2>(c, s, rec, L, k);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (s.pend >= 0) d_publish(c, s);
}

// Grid: every workgroup resident at once (tiles wait on other workgroups' tiles): one per CU.
int trunk_deep_launch(const isr_chain_desc* cd, hipStream_t s) {
    if (cd->ha % td::TH || cd->wa % td::TW || cd->nl < 1 || cd->nl > 1024) return -2;
    const long long ntiles = (long long)cd->n * (cd->wa / td::TW) * (cd->ha / td::TH);
    if (ntiles <= 0 || ntiles > (1 << 24)) return -2;
    static thread_local int cached_dev = -1, cached_per_cu = 0, cached_cus = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    const void* kern = (const void*)trunk_deep_kernel;
    if (dev != cached_dev) {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, td::LDS);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, td::NT, td::LDS) != hipSuccess) return -1;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return -1;
        cached_dev = dev;
        cached_per_cu = per_cu < 1 ? per_cu : 1;
        cached_cus = cus;
    }
    if (cached_per_cu < 1) return -4;
    const long long slots = (long long)cached_cus;
    const int grid = (int)(ntiles < slots ? ntiles : slots);
    if ((ntiles + grid - 1) / grid > td::MAX_TILES) return -2;  // the per-workgroup tile table
    const int rec_off = (int)trunk_rec_off((int)ntiles);
    if (trunk_prep_launch(cd, td::TH, s) != 0) return -1;
    hipLaunchKernelGGL(trunk_deep_kernel, dim3(grid), dim3(td::NT), td::LDS, s, cd->state, rec_off, cd->nl);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int trunk_deep_knobs_set(const int* k) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trunkd_knobs), k, 4 * sizeof(int)) == hipSuccess ? 0 : -1;
}
int trunk_deep_stamps_set(void* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trunkd_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
int trunk_deep_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trunkd_stats), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_trunkd_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#else
int trunk_deep_stats(unsigned long long*, int) { return -2; }
#endif

}  // namespace isr
