// The RRDB trunk (utils/models.py:298-317 RRDB.forward over :245-271 RDB.forward, the
// `nn.Sequential(*RRDB)` of ResNet/EResNet :598 / :627) as ONE persistent launch: every RDB
// conv (4 growth convs 64+32k -> 32 + LeakyReLU; the final 192 -> 64 conv with the RDB and
// RRDB residuals) of every block, with tile-level dependencies instead of kernel boundaries.
//
// Round-3 design.  The round-2 chain (conv3x3.hip conv_chain_kernel) ran every (layer, tile)
// as an independent conv tile: descriptor round trips, a pipeline fill, the dependency wait,
// the pipeline drain, the store drain — per tile and per layer, ~45 % of every RDB.  Here a
// workgroup runs ONE continuous stream of K-chunks over its (layer, tile) items:
//  * the 2-slot LDS ring never drains at a tile or layer boundary: the first chunk of the next
//    (layer, tile) is staged by LDS-DMA while the current tile's last chunk computes;
//  * a tile starts on the K-chunks its previous layer did NOT write (an RDB conv reads the
//    block input and the older growth outputs, which the previous layer's stencil wait already
//    covered) and waits for its 3x3 tile neighbourhood only before staging the first chunk the
//    previous layer wrote (`first_new`); that poll is issued one chunk ahead of the refill;
//  * no per-tile descriptor chain: a 64-byte layer record (compiled on the device from the
//    caller's isr_conv_desc table by trunk_prep_kernel) is read through the scalar cache, the
//    bias is staged into LDS with the first chunk;
//  * the RDB residual r1 = x[0:64] (the conv's own input) is added by four extra MFMAs per chunk
//    on the already-staged centre pixels (A = (1/s1) I, exact in bf16 for add_rate 0.2) instead
//    of re-reading 64 KB per tile in the epilogue: out = (acc + x/s1) * s1.  conv3x3.hip applies
//    the same fold at the same point of the same MFMA order, so the per-conv launches and the
//    round-2 chain stay bit-identical to this kernel.
// Hand-off (cdna_hip_programming.md Guideline 16, R1): write-through (sc1) output stores,
// drained by every wave before a workgroup barrier and a relaxed agent-scope progress store;
// consumers poll the 9 neighbour words (sc1 loads, per wave) and read activations with sc1
// LDS-DMA.  Progress words are serial numbers gen * 1024 + layers done (no zeroing per call).
#include "trunk_common.h"

namespace isr {

size_t trunk_state_words(int n, int ha, int wa) {
    const size_t tiles = (size_t)n * (ha / tk::TH) * (wa / tk::TW);
    return trunk_rec_off((int)tiles) + 1024 * 16;
}

// ---- prep: validate the layer table and compile it into records; bump the generation ----
// err bits: 1 grid, 2 view geometry, 4 kind/cout, 8 cin/bias, 16 unsupported epilogue form,
// 32 residual form, 64 a 16-channel plane of 2 GiB or more (one buffer resource spans one plane),
// 128 too many layers.
__global__ __launch_bounds__(1024) void trunk_prep_kernel(const isr_conv_desc* layers, const int32_t* kinds, int nl,
                                                          int n, int ha, int wa, unsigned* state, int th,
                                                          int h16) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    unsigned* err = reinterpret_cast<unsigned*>(smem);
    const int L = threadIdx.x;
    const int nbx = wa / tk::TW, nby = ha / th, ntiles = n * nbx * nby;
    const size_t ro = trunk_rec_off(ntiles);
    if (L == 0) *err = 0;
    __syncthreads();
    const isr_conv_desc& g0 = layers[0];
    if (L < nl) {
        const isr_conv_desc& d = layers[L];
        unsigned e = 0;
        auto same_geo = [&](const isr_view& v) {
            return v.hp == g0.x.hp && v.wp == g0.x.wp && v.cs == g0.x.cs && v.pad == g0.x.pad && v.coff % 16 == 0 &&
                   v.pad >= 1;
        };
        const int kind = kinds[L];
        // kind 2 (the training backward's RDB gather convs): a 32-cout layer whose epilogue is the
        // LeakyReLU' mask of a forward activation instead of a LeakyReLU: v = acc * (m > 0 ? 1 :
        // mslope), m = channels [m.coff, +32) of a buffer of the same geometry (no r1 / r2)
        const bool masked = kind == 2;
        if (d.n != n || d.ha != ha || d.wa != wa || d.h != g0.h || d.w != g0.w) e |= 1;
        if (!same_geo(d.x) || !same_geo(d.y) || (d.r2.data && !same_geo(d.r2)) || (masked && !same_geo(d.m))) e |= 2;
        if (kind == 0 || kind == 2 ? d.cout != 32 : (kind == 1 ? d.cout != 64 : true)) e |= 4;
        if (d.cin % 16 || d.cin < 64 || d.cin / 16 > 120 || !d.bias || ((uintptr_t)d.bias & 15)) e |= 8;
        if (d.f16 != h16 || d.shuffle != 1 || d.x_sub2 || d.taps || d.y2.data || (d.m.data != nullptr) != masked ||
            (masked && (d.m_c0 != 0 || d.slope != 1.f || d.r1.data || d.r2.data || d.s1 != 1.f || d.s2 != 1.f)))
            e |= 16;
        int fold = 0;
        uint16_t idv = 0;
        if (d.r1.data) {
            // A = (1/s1) I must be exact in the storage type (the chain's f16 flag)
            const float inv = 1.f / d.s1;
            float back;
            if (h16) {
                const _Float16 hi = (_Float16)inv;
                idv = __builtin_bit_cast(uint16_t, hi);
                back = (float)hi;
            } else {
                const __bf16 bi = (__bf16)inv;
                idv = __builtin_bit_cast(uint16_t, bi);
                back = (float)bi;
            }
            const bool alias = d.r1.data == d.x.data && d.r1.coff == d.x.coff && d.r1_cn == 0;
            if (!alias || kind != 1 || d.slope != 1.f || back != inv) e |= 32;
            fold = 1;
        } else if (d.r2.data) {
            e |= 32;
        }
        int first_new = tk::NEED_NONE;
        if (L > 0) {
            const isr_conv_desc& p = layers[L - 1];
            const int lo = p.y.coff, hi = p.y.coff + p.cout;
            first_new = d.cin / 16;  // reads nothing the previous layer wrote: wait before storing
            if (p.y.data == d.x.data) {
                for (int c = 0; c < d.cin / 16; ++c) {
                    const int c0 = d.x.coff + 16 * c;
                    if (c0 < hi && lo < c0 + 16) {
                        first_new = c;
                        break;
                    }
                }
            }
        }
        TrunkRec rec;
        rec.x = (uint64_t)(uintptr_t)d.x.data;
        rec.y = (uint64_t)(uintptr_t)d.y.data;
        rec.w = (uint64_t)(uintptr_t)d.wpack;
        rec.b = (uint64_t)(uintptr_t)d.bias;
        rec.r2 = (uint64_t)(uintptr_t)(masked ? d.m.data : d.r2.data);  // kind 2: the mask buffer
        rec.planes = (uint32_t)(d.x.coff / 16) | (uint32_t)(d.y.coff / 16) << 16;
        rec.shape = (uint32_t)((masked ? d.m.coff : d.r2.coff) / 16) | (uint32_t)(d.cin / 16) << 16 |
                    (uint32_t)(kind & 255) << 24;
        rec.deps = (uint32_t)first_new | (uint32_t)fold << 8 | (uint32_t)idv << 16;
        rec.slope = masked ? d.mslope : d.slope;
        rec.s1 = d.s1;
        rec.s2 = d.s2;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&rec);
        uint32_t* dst = state + ro + (size_t)L * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) dst[i] = src[i];
        if (e) atomicOr(err, e);
    }
    __syncthreads();
    if (L == 0) {
        const size_t plane = (size_t)g0.x.hp * g0.x.wp * 32;  // every buffer resource spans one plane
        const unsigned e = *err | (plane >= 0x7fffffffull ? 64u : 0u) | (nl > 1024 ? 128u : 0u);
        uint32_t* geo = state + ro - 16;
        const int32_t gv[16] = {n, g0.h, g0.w, ha, wa, g0.x.hp, g0.x.wp, g0.x.cs / 16, g0.x.pad, nbx, nby, ntiles,
                                (int32_t)e, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i) geo[i] = (uint32_t)gv[i];
        state[0] = state[0] + 1u;  // this launch's generation (a vector store by one lane)
    }
}

int trunk_prep_launch(const isr_chain_desc* cd, int th, hipStream_t s) {
    hipLaunchKernelGGL(trunk_prep_kernel, dim3(1), dim3(1024), 16, s, cd->layers, cd->kinds, cd->nl, cd->n, cd->ha,
                       cd->wa, cd->state, th, cd->f16 ? 1 : 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- main kernel -------------------------------------------------------------------------
#ifdef ISR_TUNING
// per (layer 75..89, tile) 8 stamps: [0] tile entry, [1] chunk 0 landed, [2] main loop done,
// [3] stores issued, [4] first dependency poll issued, [5] dependency met (s_memrealtime, 100 MHz)
__device__ unsigned long long* g_trunk_stamps;
#endif
__device__ __forceinline__ void trunk_stamp(int L, int t, int ntiles, int slot) {
#ifdef ISR_TUNING
    unsigned long long* p = g_trunk_stamps;
    if (p != nullptr && threadIdx.x == 0 && L >= 75 && L < 90) {
        unsigned long long v;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
        p[((size_t)(L - 75) * ntiles + t) * 8 + slot] = v;
    }
#else
    (void)L, (void)t, (void)ntiles, (void)slot;
#endif
}

#if ISR_TRUNK_MFMA16_PROBE
__device__ __forceinline__ f32x16 mfma32_probe16(bf16x8 a, bf16x8 b, f32x16 acc) {
    f32x4 c0 = __builtin_shufflevector(acc, acc, 0, 1, 2, 3), c1 = __builtin_shufflevector(acc, acc, 4, 5, 6, 7);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
    f32x4 c2 = __builtin_shufflevector(acc, acc, 8, 9, 10, 11), c3 = __builtin_shufflevector(acc, acc, 12, 13, 14, 15);
    f32x8 lo = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7), hi = __builtin_shufflevector(c2, c3, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
}
#endif

// Tuning builds: ablation knobs (timing only, outputs wrong): bit 1 = no halo LDS-DMA after the
// first item, 4 = no epilogue stores, 8 = no weight LDS-DMA, 16 = no dependency waits;
// [1] = workgroups per CU (host side, 0 = occupancy).  (An MFMA ablation branch inside the step
// loop would cut the MFMA/read schedule into blocks.)
#ifdef ISR_TUNING
__device__ int g_trunk_knobs[4];
static int g_trunk_per_cu = 0;
__device__ __forceinline__ int trunk_abl_load() { return __builtin_amdgcn_readfirstlane(g_trunk_knobs[0]); }
#else
__device__ __forceinline__ int trunk_abl_load() { return 0; }
#endif

// Tuning builds: per-item cycle stamps (s_memtime) for layers 77 (growth2, 8 chunks) and 79 (final,
// 12 chunks) of tile 0 of each workgroup's first tile: lane 0 of waves 0 and WM/2, 8 slots per item:
// [0] item top, [1] own DMA landed, [2] barrier passed, [3] refill issued, [4] MFMAs issued.
#ifdef ISR_TUNING
__device__ unsigned long long* g_item_stamps;
#endif
__device__ __forceinline__ void item_stamp(int L, int first_tile, int ch, int slot, int wm) {
#ifdef ISR_TUNING
    unsigned long long* p = g_item_stamps;
    const int w = wave_id();
    if (p != nullptr && first_tile && (threadIdx.x & 63) == 0 && (w == 0 || w == wm / 2) && (L == 77 || L == 79)) {
        const unsigned long long v = __builtin_amdgcn_s_memtime();
        p[((((size_t)blockIdx.x * 2 + (L == 79)) * 16 + ch) * 2 + (w != 0)) * 8 + slot] = v;
    }
#else
    (void)L, (void)first_tile, (void)ch, (void)slot, (void)wm;
#endif
}

struct TrunkArgs {
    unsigned* state;
    int rec_off;   // words
    int nl;
    int acquire;
};


// 4-byte-per-lane LDS-DMA (the bias: 64 floats = 256 B per wave instruction)
__device__ __forceinline__ void glds4(const void* gsrc, void* lds) {
    __builtin_amdgcn_global_load_lds(gsrc, ISR_LDS_PTR(lds), 4, 0, 0);
}

// One kernel build: WM waves of R output rows each (the 16-row tile), an NST-slot LDS ring (NST-1
// K-chunks in flight).  <4, 4, 2>: two 4-wave workgroups per CU, one chunk in flight (the
// round-3 first form); <8, 2, 4>: one 8-wave workgroup per CU, three chunks in flight, two tiles
// of independent images interleaved per layer.
template <int WM_, int R_, int NST_, int TH_ = 16, int XM_ = 0, int NTP_ = 0>
struct TK {
    static constexpr int WM = WM_, R = R_, NST = NST_;
    // NTP (A/B): non-temporal cache policy on the halo LDS-DMA (bit 0) / the output stores (bit 1)
    static constexpr int HALO_AUX = 16 | ((NTP_ & 1) ? 2 : 0), STORE_AUX = 16 | ((NTP_ & 2) ? 2 : 0);
    // XM = 1: XCD-aware tile deal — workgroup b (dispatched round-robin to XCD b % 8) works as
    // virtual workgroup xcd_remap(b), so each XCD streams a contiguous range of tiles and a tile's
    // halo neighbours were written through the same XCD's L2
    static constexpr int XM = XM_;
    static constexpr int NT = 64 * WM;
    static constexpr int TH = TH_;                        // tile rows (x 32 columns)
    static constexpr int HQ = (TH + 2) * tk::HC;          // halo pixels of a chunk
    static constexpr int HP = (HQ + 31) / 32;             // halo pieces (1 KB) per chunk
    static_assert(R * WM == TH, "the waves cover the tile rows");
    static_assert(NST >= 2 && NST <= 4, "ring depth");
    static constexpr int HPW = (HP + WM - 1) / WM;        // halo pieces per wave (at most)
    static constexpr int WPW = (tk::WPF + WM - 1) / WM;  // weight pieces per wave (at most)
    static constexpr int SLOT = (HP + tk::WPF) * 1024;
    static constexpr int BIAS_OFF = NST * SLOT;          // 4 bias slots of 256 B
    static constexpr int LDS = BIAS_OFF + 4 * 256;
    static_assert(LDS <= 163840, "LDS budget");
    static constexpr int BPC = 163840 / LDS < 2 ? 163840 / LDS : 2;  // workgroups per CU
    static constexpr int WPS = BPC * WM / 4;                          // waves per SIMD
    // fragment sets: 2 (the next dx step's fragments read during this step's MFMAs) or, at 4 waves
    // per SIMD (128 VGPRs), 1 — each step reads its own, the SIMD's other waves cover the latency
    static constexpr int NSET = WPS >= 4 ? 1 : 2;
};

// Where the chunks of one (layer, tile) item come from (LDS-DMA through buffer resources:
// 32-bit offsets, no per-piece 64-bit address arithmetic).
struct Src {
    const char* x;   // base of the 16-channel plane chunk 0 reads (image img, plane xp)
    uint32_t h0;     // in-plane byte offset of the halo origin: pixel (y0-1, x0-1)
    const char* w;   // packed weights of chunk 0
    const float* b;  // bias
    int wpc;         // weight pieces per chunk (9 / 18)
    uint32_t xbytes, wbytes;  // extents of one activation plane and of the packed weights
};

template <class K>
struct TrunkCtx {
    static constexpr int TH = K::TH;
    unsigned* state;
    unsigned gen;
    int acquire;
    int hp, wp, cs16, pad, h, w, nbx, nby, ntiles;
    uint32_t pstride;            // bytes per 16-channel plane (< 2 GiB: prep err bit 64); every buffer
                                 // resource spans ONE plane (a per-(image, plane) base), so the
                                 // buffers themselves may be any size (the 4K still, video batches)
    uint32_t hoff[K::HPW];       // per-lane halo piece offsets (chunk-invariant)
    int abl;                     // tuning ablation bits (0 in production builds)
};

template <class C>
__device__ __forceinline__ Src src_of(const C& c, const_rec& rec, int t) {
    const int bx = t % c.nbx, tmp = t / c.nbx, by = tmp % c.nby, img = tmp / c.nby;
    Src s;
    s.x = (const char*)(uintptr_t)rec.x + (size_t)((uint32_t)img * c.cs16 + rec_xp(rec)) * c.pstride;
    s.h0 = (uint32_t)(((by * C::TH - 1 + c.pad) * c.wp + (bx * tk::TW - 1 + c.pad)) * 32);
    s.w = (const char*)(uintptr_t)rec.w;
    s.b = (const float*)(uintptr_t)rec.b;
    s.wpc = rec_kind(rec) == 1 ? tk::WPF : tk::WPG;  // 64 / 32 couts (kinds 0 and 2: 32)
    s.xbytes = c.pstride;
    s.wbytes = (uint32_t)(rec_nch(rec) * s.wpc * 1024);
    return s;
}

// One chunk's LDS-DMA into ring slot `slot`: each wave its share of the 20 halo and 9 / 18
// weight pieces; wave 0 also the bias (first chunk of a tile).  Halo pieces are sc1 (L1
// bypass: other workgroups of this launch wrote them).  Returns the vector-memory instructions
// this wave issued (wave-uniform), for the counted waits.
template <int WM, int HPW, int WPW, int SLOTB, int BIASB, int HP, int HAUX = 16>
__device__ __forceinline__ uint32_t stage_chunk_k(const uint32_t* hoff, uint32_t pstride, int abl, const Src& s,
                                                  int chunk, int slot, bool with_bias, int bslot) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = wave_id(), lane = threadIdx.x & 63;
    char* dst = smem + slot * SLOTB;
    uint32_t n = 0;
    const auto rx = rsrc_n(s.x + (size_t)chunk * pstride, s.xbytes);  // chunk c = plane xp + c
    const uint32_t so = s.h0;
    if (!(abl & 1)) {
#pragma unroll
        for (int k = 0; k < HPW; ++k) {
            const int j = wave + WM * k;
            if (j < HP) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, ISR_LDS_PTR(dst + j * 1024), 16, hoff[k], so, 0, HAUX);
                ++n;
            }
        }
    }
    const auto rw = rsrc_n(s.w, s.wbytes);
    const uint32_t wo = (uint32_t)(chunk * s.wpc * 1024);
    char* wd = dst + HP * 1024;
#pragma unroll
    for (int k = 0; k < WPW; ++k) {
        const int j = wave + WM * k;
        if (j < s.wpc && !(abl & 8)) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, ISR_LDS_PTR(wd + j * 1024), 16, lane * 16, wo + j * 1024, 0, 0);
            ++n;
        }
    }
    if (with_bias && wave == 0) {
        if (lane < (s.wpc == tk::WPG ? 32 : 64))  // cout floats only
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n(s.b, s.wpc == tk::WPG ? 128u : 256u), ISR_LDS_PTR(smem + BIASB + bslot * 256), 4,
                                                     lane * 4, 0, 0, 0);
        ++n;
    }
    return n;
}

template <class K>
__device__ __forceinline__ uint32_t stage_chunk(const TrunkCtx<K>& c, const Src& s, int chunk, int slot, bool with_bias,
                                                int bslot) {
#ifdef ISR_TUNING
    // tuning-build check of the ring protocol: the chunk lies inside the layer (chunk < nch: its
    // weights inside the packed table) and the slot inside the ring.  A violation gives the launch
    // up (the host raises) and issues nothing, instead of a DMA to a wrong place.
    if (chunk < 0 || (uint32_t)(chunk * s.wpc * 1024) >= s.wbytes || slot < 0 || slot >= K::NST ||
        bslot < 0 || bslot > 3) {
        if (threadIdx.x == 0) {
            __hip_atomic_store(c.state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(c.state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return 0;
    }
#endif
    if constexpr (K::NSET == 1) {
        // the 128-VGPR form: the per-lane halo offsets rebuilt from an opaque lane id per chunk
        // (kept live they spilled, and a scratch reload's vmcnt wait would drain the ring's DMA)
        int ln = threadIdx.x & 63;
        asm volatile("" : "+v"(ln));
        uint32_t ho[K::HPW];
#pragma unroll
        for (int k = 0; k < K::HPW; ++k) ho[k] = halo_piece_off<K::HQ>(wave_id() + K::WM * k, ln, c.wp);
        return stage_chunk_k<K::WM, K::HPW, K::WPW, K::SLOT, K::BIAS_OFF, K::HP, K::HALO_AUX>(ho, c.pstride, c.abl, s, chunk, slot,
                                                                          with_bias, bslot);
    }
    return stage_chunk_k<K::WM, K::HPW, K::WPW, K::SLOT, K::BIAS_OFF, K::HP, K::HALO_AUX>(c.hoff, c.pstride, c.abl, s, chunk, slot,
                                                                      with_bias, bslot);
}

// Interleaved refill (the pair form's one refill item issued one piece per MFMA of step 0 or, with
// -DISR_TRUNK_INTERLEAVE=2, of step 2): OFF.  Bit-identical (tests/test_gpu_chain.py) but slower:
// 7.41 / 7.47 ms per bench forward against 6.64 ms for the block issue, same box, two rounds each
// (profiles/r03_trunk_interleave_ab.jsonl) — the LDS-DMA issue stalls the wave's in-order MFMA
// stream wherever it sits, so spreading it only adds the stalls to the matrix-pipe chain.  This
// build (python -m image_super_resolution_amd._build --interleave) passes tests/test_gpu_chain.py
// bit for bit (round 4).  Round 3's first version also deferred EVERY staged item by one loop
// pass and re-derived the deferred item's chunk and slot as (so - h0) / pstride and
// (dst - smem) / SLOT; that run gave wrong 8-wave outputs and faulted the card once.  Both
// re-derivations are exact (so = h0 + chunk * pstride with the tile offset below one plane, dst =
// smem + slot * SLOT), the pieces stay inside a slot in both forms and push_mark's positions
// follow the issue order, so no chunk, slot or offset of that diff can be shown out of range
// from the code; the run was not repeated.  The bug class is closed instead: every buffer
// resource carries its tensor's real extent (rsrc_n: an offset past it reads zeros / drops the
// store), and the tuning build checks chunk < nch, slot < NST and the bias slot before issuing.
// Wave priority: 1 (production) raises the wave to priority 1 around each chunk's MFMA stream
// (s_setprio, cdna_hip_programming.md T5), so the co-resident workgroup's refill / epilogue issue
// yields to it: 6.567 / 6.566 vs 6.620 / 6.592 ms per bench forward, same box, two rounds
// (profiles/r03_trunk_prio_ab.jsonl); 2 (a static priority for the later-dispatched half of the
// grid) measured no change; 0 = none.
#ifndef ISR_TRUNK_PRIO
#define ISR_TRUNK_PRIO 1
#endif
// 1: the refill's LDS-DMA issued before the step-0 fragment reads instead of after them (the DMA
// issue is cheaper with no reads in flight, MI355X_MICROARCH.md): a tie, 6.598 / 6.598 / 6.575
// vs 6.558 / 6.609 / 6.583 ms (profiles/r03_trunk_refill_order_ab.jsonl) — kept off.
#ifndef ISR_TRUNK_REFILL_FIRST
#define ISR_TRUNK_REFILL_FIRST 0
#endif
constexpr bool kRefillFirst = ISR_TRUNK_REFILL_FIRST != 0;
#ifndef ISR_TRUNK_INTERLEAVE
#define ISR_TRUNK_INTERLEAVE 0
#endif
constexpr bool kTrunkInterleave = ISR_TRUNK_INTERLEAVE != 0;
// the step (dx) whose MFMAs carry the pieces: 0 (interleave 1) or 2 (interleave 2: after the
// chunk's last LDS fragment read, so no later read of this chunk can be held behind the DMA)
constexpr int kTrunkInterleaveStep = ISR_TRUNK_INTERLEAVE == 2 ? 2 : 0;

// A refill whose LDS-DMA pieces are issued one per MFMA of the next step instead of in one block
// before the MFMAs (a block of 7-11 LDS-DMA issues per wave ran ~1,000-2,600 cycles with the
// matrix pipe idle: tools/trunk_items.py "reads+refill").  Same pieces, same count, same slots.
struct Refill {
    bool on;
    Src src;
    const char* xb;    // the chunk's plane base
    uint32_t so, wo;   // in-plane halo offset of the chunk, weight offset
    char* dst;         // slot base in LDS
    bool bias;
    int bslot;
};

// Piece p of this wave's share (p < HPW: halo, then weights, then the bias); p is a constant
// once the MFMA loop it is called from is unrolled.
template <int WM, int HPW, int WPW, int BIASB, int HP>
__device__ __forceinline__ uint32_t refill_piece_k(const uint32_t* hoff, int abl, const Refill& rf, const int p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = wave_id(), lane = threadIdx.x & 63;
    if (p < HPW) {
        const int j = wave + WM * p;
        if (!(abl & 1) && j < HP) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n(rf.xb, rf.src.xbytes), ISR_LDS_PTR(rf.dst + j * 1024), 16, hoff[p],
                                                     rf.so, 0, 16);
            return 1;
        }
        return 0;
    }
    if (p < HPW + WPW) {
        const int j = wave + WM * (p - HPW);
        if (j < rf.src.wpc) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n(rf.src.w, rf.src.wbytes), ISR_LDS_PTR(rf.dst + (HP + j) * 1024), 16,
                                                     lane * 16, rf.wo + j * 1024, 0, 0);
            return 1;
        }
        return 0;
    }
    if (p == HPW + WPW && rf.bias && wave == 0) {
        if (lane < (rf.src.wpc == tk::WPG ? 32 : 64))  // cout floats only
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_n(rf.src.b, rf.src.wpc == tk::WPG ? 128u : 256u), ISR_LDS_PTR(smem + BIASB + rf.bslot * 256), 4,
                                                     lane * 4, 0, 0, 0);
        return 1;
    }
    return 0;
}

template <class K>
__device__ __forceinline__ uint32_t refill_piece(const TrunkCtx<K>& c, const Refill& rf, const int p) {
    return refill_piece_k<K::WM, K::HPW, K::WPW, K::BIAS_OFF, K::HP>(c.hoff, c.abl, rf, p);
}

template <class K>
__device__ __forceinline__ Refill make_refill(const TrunkCtx<K>& c, const Src& s, int chunk, int slot, bool with_bias,
                                              int bslot) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Refill rf;
    rf.on = true;
    rf.src = s;
    rf.xb = s.x + (size_t)chunk * c.pstride;
    rf.so = s.h0;
    rf.wo = (uint32_t)(chunk * s.wpc * 1024);
    rf.dst = smem + slot * K::SLOT;
    rf.bias = with_bias;
    rf.bslot = bslot;
#ifdef ISR_TUNING
    if (chunk < 0 || rf.wo >= s.wbytes || slot < 0 || slot >= K::NST || bslot < 0 || bslot > 3) {
        if (threadIdx.x == 0) {  // as in stage_chunk: give the launch up, issue nothing
            __hip_atomic_store(c.state + 1, c.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(c.state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        rf.on = false;
    }
#endif
    return rf;
}

// The tile that follows the current one in this workgroup's stream.
struct Next {
    bool exists;
    int L, t;
    Src src;
    int first_new;   // its first chunk its previous layer wrote (NEED_NONE on layer 0)
    int nch;
    bool self_dep;   // its neighbourhood contains the tile being computed now
};

// Per wave, carried from item to item (all wave-uniform).  Items are the K-chunks of the
// stream in order; `issued` counts this wave's vector-memory instructions, and m[0..] holds
// `issued` right after the DMA of the current item and of the items staged after it, so the
// top of an item waits for exactly its own DMA (wait_vm(issued - m[0])) and leaves the later
// items, stores and loads in flight.
template <class K>
struct Stream {
    int item;             // global index of the item being computed
    int staged;           // global index of the last item whose DMA was issued
    int tseq;             // tiles started (bias slot = tseq & 3)
    uint32_t issued;
    uint32_t m0, m1, m2, m3;  // FIFO: m0 = current item (named scalars: an array would be indexed
                              // at run time and live in scratch, whose ops count in vmcnt)
    int pend_t;           // tile whose progress word waits for its stores (-1: none)
    unsigned pend_v;
    uint32_t pend_mark;   // `issued` right after those stores
    bool dep_next;        // the next tile's neighbourhood has been verified
};

template <class K>
__device__ __forceinline__ void push_mark(Stream<K>& st) {
    const int pos = st.staged - st.item;  // position of the item just staged
    const uint32_t v = st.issued;
    st.m0 = pos == 0 ? v : st.m0;
    st.m1 = pos == 1 ? v : st.m1;
    st.m2 = pos == 2 ? v : st.m2;
    st.m3 = pos >= 3 ? v : st.m3;
}

template <class K>
__device__ __forceinline__ void pop_mark(Stream<K>& st) {
    st.m0 = st.m1;
    st.m1 = st.m2;
    st.m2 = st.m3;
}

// Publish the pending tile's progress word now (every wave drains all its vector memory, then a
// workgroup barrier): required before any blocking wait, so that no workgroup ever spins on a
// word this workgroup holds back.  Wave-uniform call sites only (it contains a barrier).
template <class K>
__device__ __forceinline__ void force_publish(const TrunkCtx<K>& c, Stream<K>& st) {
    if (st.pend_t < 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    if (threadIdx.x == 0)
        __hip_atomic_store(c.state + 4 + st.pend_t, st.pend_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st.pend_t = -1;
}

template <class K, int NF, bool MASKED = false, bool H = false>
__device__ __forceinline__ void run_tile(const TrunkCtx<K>& c, Stream<K>& st, const_rec& rec, int L, int t,
                                         const Next& nx) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int R = K::R, NST = K::NST, CT = 32 * NF, TN = 3, NA = R + 2;
    const int wave = wave_id(), lane = threadIdx.x & 63, l31 = lane & 31, hh = lane >> 5;
    const int bx = t % c.nbx, tmp = t / c.nbx, by = tmp % c.nby, img = tmp / c.nby;
    const int x0 = bx * tk::TW, y0 = by * K::TH;
    const int nch = rec_nch(rec);
    const int first_new = rec_first_new(rec);  // NEED_NONE on layer 0
    const unsigned need = c.gen * 1024u + (unsigned)L;  // the neighbourhood is done with layer L-1
    const bool fold = NF == 2 && rec_fold(rec);
    const bool has_r2 = NF == 2 && rec.r2 != 0;
    constexpr bool masked = NF == 1 && MASKED;  // kind 2 (gather conv): LeakyReLU' mask from rec.r2
    const Src me = src_of(c, rec, t);
    bool dep_ok = first_new == tk::NEED_NONE || st.dep_next;
    st.dep_next = false;
    const int bslot = st.tseq & 3;
    const int first_item = st.item;  // this tile's chunk 0
    trunk_stamp(L, t, c.ntiles, 0);

    // per-lane LDS read addresses (slot 0): weights A[n][k] (n = cout), halo rows of this wave
    const uint32_t a_w = (uint32_t)(K::HP * 1024 + (2 * l31 + (hh ^ ((l31 >> 3) & 1))) * 16);
    uint32_t a_h[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
        a_h[dx] = (uint32_t)((wave * R * tk::HC + l31 + dx) * 32 + 16 * (hh ^ (((l31 + dx) >> 3) & 1)));

    // neighbourhood wait (blocking), preceded by the pending publish
    auto wait_deps = [&](int tt, unsigned nd) {
        force_publish(c, st);
        trunk_stamp(L, t, c.ntiles, 4);
        if (!(c.abl & 16)) dep_wait(c.state, nb_of(tt, c.nbx, c.nby), nd, c.gen);
        if (c.acquire) acquire_fence();
        trunk_stamp(L, t, c.ntiles, 5);
    };

    f32x16 acc[R][NF];

    // one K-chunk; FC = the chunk index (0..3) when the residual fold adds its MFMAs to it, else -1
    // (peeled so that the fold's target accumulator is compile-time: a run-time choice made hipcc
    // MFMA into a temporary and copy 16 VGPRs back)
    const uint32_t idv = rec_idv(rec);
    auto do_chunk = [&](const int ch, auto fc_tag) {
        constexpr int FC = decltype(fc_tag)::value;
            const int slot = st.item % NST;
            const bool stamp_tile = t == (int)blockIdx.x;
            item_stamp(L, stamp_tile, ch, 0, K::WM);
            // ---- top of item: this item's DMA has landed for every wave ----
            if (st.staged < st.item) {
                // not staged (the next tile needed this tile's own outputs): drain, publish, wait, stage
                force_publish(c, st);
                if (ch >= first_new && !dep_ok) {
                    wait_deps(t, need);
                    dep_ok = true;
                }
                st.issued += stage_chunk(c, me, ch, slot, ch == 0, bslot);
                st.staged = st.item;
                push_mark(st);
            }
            wait_vm(st.issued - st.m0);
            item_stamp(L, stamp_tile, ch, 1, K::WM);
            raw_barrier();
            item_stamp(L, stamp_tile, ch, 2, K::WM);
            if (st.pend_t >= 0 && (int)(st.m0 - st.pend_mark) >= 0) {  // its stores are older than this DMA
                if (threadIdx.x == 0)
                    __hip_atomic_store(c.state + 4 + st.pend_t, st.pend_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                st.pend_t = -1;
            }
            if (ch == 0) {
                trunk_stamp(L, t, c.ntiles, 1);
                // bias → accumulators (register g of lane l: cout (g&3) + 8(g>>2) + 4hh of fragment f)
                const float* bs = reinterpret_cast<const float*>(smem + K::BIAS_OFF + bslot * 256);
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
            const char* sb = smem + slot * K::SLOT;
            constexpr int NSET = K::NSET;
            // the 1-set (128-VGPR) form rebuilds its fragment addresses from an opaque lane id at
            // each chunk: kept live across the chunks, they were what it spilled
            uint32_t aw = a_w, ah[3] = {a_h[0], a_h[1], a_h[2]};
            if constexpr (NSET == 1) {
                int ln = threadIdx.x & 63;
                asm volatile("" : "+v"(ln));
                const int q31 = ln & 31, qh = ln >> 5;
                aw = (uint32_t)(K::HP * 1024 + (2 * q31 + (qh ^ ((q31 >> 3) & 1))) * 16);
    #pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    ah[dx] = (uint32_t)((wave * R * tk::HC + q31 + dx) * 32 + 16 * (qh ^ (((q31 + dx) >> 3) & 1)));
            }
            bf16x8 fb[NSET][TN][NF], fa[NSET][NA];
            auto read_one = [&](int dx, int idx, int set) {
                if (idx < TN * NF) {
                    const int dyi = idx / NF, f = idx % NF;
                    fb[set][dyi][f] = lds_read16(sb + aw + ((dyi * 3 + dx) * CT * 2 + f * 64) * 16);
                } else {
                    const int ia = idx - TN * NF;
                    fa[set][ia] = lds_read16(sb + ah[dx] + ia * tk::HC * 32);
                }
            };
            auto read_fb = [&](int dx, int dyi, int set) {
    #pragma unroll
                for (int f = 0; f < NF; ++f) read_one(dx, dyi * NF + f, set);
            };
            // step 0's fragments in order of first use (kernel-row-major MFMA order below); with
            // ISR_TRUNK_REFILL_FIRST the refill's LDS-DMA is issued before them instead of after
            auto read_step0 = [&]() {
                if constexpr (K::NSET == 1) {  // lazy: kernel row 0's weights and its R input rows
                    read_fb(0, 0, 0);
    #pragma unroll
                    for (int ia = 0; ia < R; ++ia) read_one(0, TN * NF + ia, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    return;
                }
                read_fb(0, 0, 0);
    #pragma unroll
                for (int ia = 0; ia < R; ++ia) read_one(0, TN * NF + ia, 0);
                read_fb(0, 1, 0);
                read_one(0, TN * NF + R, 0);
                read_fb(0, 2, 0);
                read_one(0, TN * NF + R + 1, 0);
                __builtin_amdgcn_sched_barrier(0);
            };
            if constexpr (!kRefillFirst) read_step0();

            // ---- refill: stage the stream up to NST-1 items ahead (own chunks, then the next tile's).
            // The last item to stage is deferred: its pieces go out one per MFMA of step 0 below
            // (an earlier one in the same pass is issued at once, when a later one follows). ----
            Refill rf;
            rf.on = false;
            while (st.staged < st.item + NST - 1) {
                const int off = st.staged + 1 - first_item;  // chunk offset from this tile's chunk 0
                const int nslot = (st.staged + 1) % NST;
                if (off < nch) {
                    if (off >= first_new && !dep_ok) {
                        wait_deps(t, need);
                        dep_ok = true;
                    }
                    if constexpr (kTrunkInterleave && NST == 2) {
                        if (st.staged + 1 == st.item + NST - 1) {  // the last item of this pass: deferred
                            rf = make_refill(c, me, off, nslot, false, 0);
                            ++st.staged;
                            break;
                        }
                    }
                    st.issued += stage_chunk(c, me, off, nslot, false, 0);
                } else {
                    const int nc = off - nch;
                    if (!nx.exists || nc >= nx.nch) break;
                    if (nx.L > 0 && nc >= nx.first_new && !st.dep_next) {
                        if (nx.self_dep) break;  // needs this tile's outputs: staged at its own top
                        wait_deps(nx.t, c.gen * 1024u + (unsigned)nx.L);
                        st.dep_next = true;
                    }
                    if constexpr (kTrunkInterleave && NST == 2) {
                        if (st.staged + 1 == st.item + NST - 1) {
                            rf = make_refill(c, nx.src, nc, nslot, nc == 0, (bslot + 1) & 3);
                            ++st.staged;
                            break;
                        }
                    }
                    st.issued += stage_chunk(c, nx.src, nc, nslot, nc == 0, (bslot + 1) & 3);
                }
                ++st.staged;
                push_mark(st);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (kRefillFirst) read_step0();
            item_stamp(L, stamp_tile, ch, 3, K::WM);
            uint32_t rf_n = 0;
#if ISR_TRUNK_PRIO == 1
            __builtin_amdgcn_s_setprio(1);  // the MFMA stream ahead of the partner's issue
#endif

            // ---- MFMAs: 3 steps (dx), each in kernel-row-major order (dy, then output row r):
            // every accumulator still sees dy 0, 1, 2 in that order (conv3x3.hip's input-row-major
            // loop gives each accumulator the same sequence, so the bits agree).  The next step's
            // fragment of kernel row dy is read right after that row's last MFMA here, and its
            // input row ia right after the current one's last use. ----
    #pragma unroll
            for (int stp = 0; stp < 3; ++stp) {
                const int cur = NSET == 2 ? (stp & 1) : 0;
                if constexpr (NSET == 1) {
                    if (stp > 0) {  // lazy: kernel row 0's weights and the first R input rows
                        read_fb(stp, 0, 0);
    #pragma unroll
                        for (int ia = 0; ia < R; ++ia) read_one(stp, TN * NF + ia, 0);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
    #pragma unroll
                for (int dyi = 0; dyi < TN; ++dyi) {
                    if constexpr (NSET == 1) {
                        // the next kernel row's weights and its one new input row, one row ahead:
                        // at most two kernel rows' fragments are live (the 128-VGPR budget)
                        if (dyi + 1 < TN) {
                            read_fb(stp, dyi + 1, 0);
                            read_one(stp, TN * NF + dyi + R, 0);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
    #pragma unroll
                    for (int r = 0; r < R; ++r) {
#if ISR_TRUNK_MFMA16_PROBE
                        // timing probe (lib/libisr_probe16.so, outputs wrong): each growth-chunk
                        // 32x32x16 MFMA replaced by two 16x16x32 of the same FLOPs on the same operands
                        if constexpr (NF == 1) {
                            acc[r][0] = mfma32_probe16(fb[cur][dyi][0], fa[cur][r + dyi], acc[r][0]);
                        } else
#endif
    #pragma unroll
                        for (int f = 0; f < NF; ++f) acc[r][f] = mfma32t<H>(fb[cur][dyi][f], fa[cur][r + dyi], acc[r][f]);
                        if constexpr (NF == 2 && FC >= 0) {
                            // residual fold: + x/s1 on the centre pixels of row r (dx = 1, dy = 1),
                            // between the row's dy = 1 and dy = 2 contributions (chunk FC, compile-time)
                            if (dyi == 1 && stp == 1) {
                                const bf16x8 a = fold_a_bits<K::NSET == 1>(idv, FC & 1);
                                acc[r][FC >> 1] = mfma32t<H>(a, fa[cur][r + 1], acc[r][FC >> 1]);
                            }
                        }
                        // input row ia = r + dyi is last used here when dyi == min(2, ia)
                        if (NSET == 2 && stp + 1 < 3 && (dyi == 2 || r == 0))
                            read_one(stp + 1, TN * NF + r + dyi, cur ^ 1);
                        if (stp == kTrunkInterleaveStep && rf.on) rf_n += refill_piece<K>(c, rf, dyi * R + r);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (NSET == 2 && stp + 1 < 3) {
                        read_fb(stp + 1, dyi, cur ^ 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if (stp == kTrunkInterleaveStep && rf.on) {
                    // pieces beyond step 0's MFMA count (the 8-wave form), then the item's mark
    #pragma unroll
                    for (int q = TN * R; q <= K::HPW + K::WPW; ++q) rf_n += refill_piece<K>(c, rf, q);
                    st.issued += rf_n;
                    push_mark(st);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#if ISR_TRUNK_PRIO == 1
            __builtin_amdgcn_s_setprio(0);
#endif
            item_stamp(L, stamp_tile, ch, 4, K::WM);
            pop_mark(st);  // the FIFO head moves to the next item (marks are positions from st.item)
    };
    int ch0 = 0;
    if constexpr (NF == 2) {
        if (fold && nch >= 4) {
            do_chunk(0, TIC<0>{});
            ++st.item;
            do_chunk(1, TIC<1>{});
            ++st.item;
            do_chunk(2, TIC<2>{});
            ++st.item;
            do_chunk(3, TIC<3>{});
            ++st.item;
            ch0 = 4;
        }
    }
    for (int ch = ch0; ch < nch; ++ch, ++st.item) do_chunk(ch, TIC<-1>{});
    trunk_stamp(L, t, c.ntiles, 2);

    // the neighbourhood must be done with layer L-1 before this tile's outputs land (a layer
    // that reads nothing its predecessor wrote never waited above)
    if (!dep_ok && first_new != tk::NEED_NONE) wait_deps(t, need);

    // ---- epilogue: straight from the accumulators, write-through (sc1) stores ----
    {
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const int xx = x0 + l31;
        const float slope = rec.slope, s1 = rec.s1, s2 = rec.s2;
        const bool scale2 = s2 != 1.f;
        // one buffer resource per output plane (cout channels = NF * 2 planes of 16): couts
        // [32 f + 16 blk, + 16) live in plane yp + 2 f + blk of image img
        const char* ybase = (const char*)(uintptr_t)rec.y + (size_t)((uint32_t)img * c.cs16 + rec_yp(rec)) * c.pstride;
        // RRDB residual (every third RDB's final conv): row r + 1's values are loaded while row r
        // is finished, so at most two rows (32 VGPRs) are live — loading them all before the last
        // chunk's MFMAs (64 VGPRs beside the 128 accumulators and the fragments) spilled.
        // Compiler-visible loads: hipcc places the wait before their first use itself.
        bf16x8 q2[R][NF][2];
        const char* r2base = (const char*)(uintptr_t)rec.r2 + (size_t)((uint32_t)img * c.cs16 + rec_r2p(rec)) * c.pstride;
        auto load_r2 = [&](int r) {
            const uint32_t pix = (uint32_t)((y0 + wave * R + r + c.pad) * c.wp + xx + c.pad);
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const auto rr = rsrc_n(r2base + (size_t)(2 * f + blk) * c.pstride, c.pstride);
                    q2[r][f][blk] = __builtin_bit_cast(
                        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rr, pix * 32 + 16 * hh, 0, 16));
                }
            st.issued += NF * 2;
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
                            u[e] = elt<H>(q2[r][f][blk], e) > 0.f ? u[e] : u[e] * slope;
                        else
                            u[e] = u[e] >= 0.f ? u[e] : u[e] * slope;
                        if (fold) u[e] = u[e] * s1;
                        if (has_r2) {
                            u[e] = u[e] * s2 + elt<H>(q2[r][f][blk], e);
                        } else {
                            if (scale2) u[e] *= s2;
                        }
                        if (!valid) u[e] = 0.f;
                    }
                    const auto yr = rsrc_n(ybase + (size_t)(2 * f + blk) * c.pstride, c.pstride);
                    const uint32_t off = pix * 32 + 16 * hh;
                    const bf16x8 tq = pack8<H>(u);
                    if (!(c.abl & 4)) {
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tq), yr, off, 0, K::STORE_AUX);
                        ++st.issued;
                    }
                }
            }
        }
    }
    trunk_stamp(L, t, c.ntiles, 3);
    st.pend_t = t;
    st.pend_v = c.gen * 1024u + (unsigned)(L + 1);
    st.pend_mark = st.issued;
    ++st.tseq;
}

template <class K, bool H = false>
__global__ __launch_bounds__(K::NT, K::WPS) void trunk_kernel(TrunkArgs a) {
    TrunkCtx<K> c;
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
    c.abl = trunk_abl_load();
    {
        const int wave = wave_id(), lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < K::HPW; ++k) c.hoff[k] = K::NSET == 1 ? 0u : halo_piece_off<K::HQ>(wave + K::WM * k, lane, c.wp);
    }
    const int G = gridDim.x, b = K::XM ? xcd_remap((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
#if ISR_TRUNK_PRIO == 2
    // tuning A/B: the later-dispatched half of the grid (a CU's second workgroup) at priority 1
    if (__builtin_amdgcn_readfirstlane(b) >= G / 2) __builtin_amdgcn_s_setprio(1);
#endif
    Stream<K> st;
    st.item = 0;
    st.staged = 0;
    st.tseq = 0;
    st.issued = 0;
    st.m0 = st.m1 = st.m2 = st.m3 = 0;
    st.pend_t = -1;
    st.pend_v = 0;
    st.pend_mark = 0;
    st.dep_next = false;
    if (b < c.ntiles) {
        st.issued += stage_chunk(c, src_of(c, recs[0], b), 0, 0, true, 0);  // layer 0 reads the trunk input only
        st.m0 = st.issued;
        for (int L = 0; L < a.nl; ++L) {
            const_rec& rec = recs[L];
            for (int t = b; t < c.ntiles; t += G) {
                Next nx;
                nx.exists = true;
                if (t + G < c.ntiles) {
                    nx.L = L;
                    nx.t = t + G;
                } else if (L + 1 < a.nl) {
                    nx.L = L + 1;
                    nx.t = b;
                } else {
                    nx.exists = false;
                    nx.L = L;
                    nx.t = t;
                }
                const_rec& nrec = recs[nx.L];
                nx.src = src_of(c, nrec, nx.t);
                nx.first_new = rec_first_new(nrec);
                nx.nch = rec_nch(nrec);
                {
                    const int bx = t % c.nbx, tq = t / c.nbx, by = tq % c.nby, im = tq / c.nby;
                    const int bx2 = nx.t % c.nbx, nq = nx.t / c.nbx, by2 = nq % c.nby, im2 = nq / c.nby;
                    nx.self_dep = im == im2 && abs(bx - bx2) <= 1 && abs(by - by2) <= 1;
                }
                const int kind = rec_kind(rec);
                if (kind == 0) run_tile<K, 1, false, H>(c, st, rec, L, t, nx);
                else if (kind == 2) run_tile<K, 1, true, H>(c, st, rec, L, t, nx);  // the backward chain's gathers
                else run_tile<K, 2, false, H>(c, st, rec, L, t, nx);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && st.pend_t >= 0)
        __hip_atomic_store(c.state + 4 + st.pend_t, st.pend_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid: every workgroup must be resident at once (tiles wait on other workgroups' tiles), so
// the grid is min(tiles, resident workgroups) with residency from the occupancy API (capped at
// what the build is made for); ISR_ERR when that is below one workgroup per CU.
template <class K, bool H = false>
static int trunk_launch_k(const isr_chain_desc* cd, hipStream_t s) {
    if (cd->ha % K::TH || cd->wa % tk::TW || cd->nl < 1 || cd->nl > 1024) return -2;
    const int nbx = cd->wa / tk::TW, nby = cd->ha / K::TH;
    const long long ntiles = (long long)cd->n * nbx * nby;
    if (ntiles <= 0 || ntiles > (1 << 24)) return -2;
    static thread_local int cached_dev = -1, cached_per_cu = 0, cached_cus = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    const void* kern = (const void*)trunk_kernel<K, H>;
    if (dev != cached_dev) {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, K::NT, K::LDS) != hipSuccess) return -1;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return -1;
        cached_dev = dev;
        cached_per_cu = per_cu < K::BPC ? per_cu : K::BPC;
        cached_cus = cus;
    }
    int per_cu = cached_per_cu;
#ifdef ISR_TUNING
    if (g_trunk_per_cu > 0 && g_trunk_per_cu < per_cu) per_cu = g_trunk_per_cu;
#endif
    if (per_cu < 1) return -4;
    const long long slots = (long long)per_cu * cached_cus;
    const int grid = (int)(ntiles < slots ? ntiles : slots);
    const int rec_off = (int)trunk_rec_off((int)ntiles);
    trunk_prep_launch(cd, K::TH, s);
    TrunkArgs a;
    a.state = cd->state;
    a.rec_off = rec_off;
    a.nl = cd->nl;
    a.acquire = cd->acquire;
    hipLaunchKernelGGL((trunk_kernel<K, H>), dim3(grid), dim3(K::NT), K::LDS, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// production: two 4-wave workgroups per CU, one chunk in flight (237 VGPRs, no scratch since
// the RRDB residual is loaded row by row in the epilogue): 6.46 ms per bench forward against
// 7.77 ms for the deep form (same box, tools/ab_chain.py, profiles/r03_ab_chain.jsonl) — the deep
// form's 2-row waves read 7 LDS fragments per 6 MFMAs (4-row waves: 9 per 12)
// ISR_TRUNK_XCD=1 (A/B build lib/libisr_xcd.so, _build.build_trunk_alt): the same form with the
// XCD-aware tile deal (each XCD streams a contiguous range of tiles; bit-identical outputs)
#ifndef ISR_TRUNK_XCD
#define ISR_TRUNK_XCD 0
#endif
using TK_PAIR = TK<4, 4, 2, 16, ISR_TRUNK_XCD>;

// The A/B forms below measured slower than the pair form on the same boxes and are
// compiled only into the tuning library (-DISR_TUNING, lib/libisr_tuning.so): the production
// libisr.so carries the production form alone.
#ifdef ISR_TUNING
using TK_DEEP = TK<8, 2, 4>;   // one 8-wave workgroup per CU, 3 chunks in flight
// 32x32 tiles: one 8-wave workgroup per CU (4 rows per wave, as the pair form), the chunk's
// weights staged once per CU instead of twice and a (34x34)/(32x32) halo instead of (18x34)/(16x32)
using TK_T32 = TK<8, 4, 2, 32>;
// the pair form's tile, ring and two workgroups per CU with 8 waves each (2 rows per wave): 4 waves
// per SIMD at 128 VGPRs (one fragment set), and each wave issues half the refill pieces
using TK_QUAD = TK<8, 2, 2>;
using TK_PAIR_X = TK<4, 4, 2, 16, 1>;  // the pair form with the XCD-aware tile deal
using TK_PAIR_NTH = TK<4, 4, 2, 16, 0, 1>;  // non-temporal halo loads
using TK_PAIR_NTS = TK<4, 4, 2, 16, 0, 2>;  // non-temporal output stores
// (round 6: the deep-ring form of trunk_deep.hip and the loader / consumer form of trunk_lc.hip,
// chain variants 4 and 9, measured slower in rounds 4-5 — DESIGN.md §5 — and were removed)
#endif

int trunk_launch(const isr_chain_desc* cd, hipStream_t s, int form) {
    if (cd->f16) return form == 0 ? trunk_launch_k<TK_PAIR, true>(cd, s) : -3;  // fp16 storage: production form only
    if (form == 0) return trunk_launch_k<TK_PAIR>(cd, s);
#ifdef ISR_TUNING
    if (form == 2) return trunk_launch_k<TK_T32>(cd, s);
    if (form == 4) return trunk_launch_k<TK_QUAD>(cd, s);
    if (form == 5) return trunk_launch_k<TK_PAIR_X>(cd, s);
    if (form == 6) return trunk_launch_k<TK_PAIR_NTH>(cd, s);
    if (form == 7) return trunk_launch_k<TK_PAIR_NTS>(cd, s);
    if (form == 1) return trunk_launch_k<TK_DEEP>(cd, s);
#endif
    return -3;  // an A/B form of the tuning library
}

#ifdef ISR_TUNING
int trunk_knobs_set(const int* k) {
    g_trunk_per_cu = k[1];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trunk_knobs), k, 4 * sizeof(int)) == hipSuccess ? 0 : -1;
}
int trunk_stamps_set(void* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_trunk_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1; }
int trunk_item_stamps_set(void* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_item_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#else
int trunk_knobs_set(const int*) { return -2; }
int trunk_stamps_set(void*) { return -2; }
int trunk_item_stamps_set(void*) { return -2; }
#endif

}  // namespace isr
