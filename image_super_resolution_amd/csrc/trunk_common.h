// Shared pieces of the persistent RRDB-trunk kernels (trunk.hip: the two-workgroups-per-CU pair
// form and its variants; until round 6 also trunk_deep.hip): layer records, the
// dependency poll, buffer resources, the LDS halo image, counted vmcnt waits.
#pragma once
#include "isr_common.h"

namespace isr {

namespace tk {
constexpr int TH = 16;          // tile rows (R x WM of a build)
constexpr int TW = 32;
constexpr int HR = TH + 2, HC = TW + 2, HQ = HR * HC;  // 18 x 34 halo pixels
constexpr int HP = (HQ + 31) / 32;                      // 20 halo pieces (1 KB) per chunk
constexpr int WPG = 9, WPF = 18;                        // weight pieces per chunk: 32 / 64 couts
constexpr int NEED_NONE = 255;
}  // namespace tk

// Layer record (64 bytes at state words [rec_off + 16 L, + 16)), dwords only: a scalar load
// cannot fetch bytes on gfx950, so packed small fields are unpacked with scalar shifts.
struct TrunkRec {
    uint64_t x, y, w, b, r2;   // buffer bases, packed weights, fp32 bias, r2 base (or 0)
    uint32_t planes;           // xp | yp << 16: first 16-channel plane of x / y (coff / 16)
    uint32_t shape;            // r2p | nch << 16 | kind << 24 (nch = cin / 16; kind 0 growth, 1 final)
    uint32_t deps;             // first_new | fold << 8 | idv << 16 (first chunk the previous layer
                               // wrote, NEED_NONE on layer 0; fold: r1 == x[0:cout] added as x/s1
                               // by MFMA; idv: bf16 bits of 1/s1)
    float slope, s1, s2;
};
static_assert(sizeof(TrunkRec) == 64, "record size");

// Geometry (16 words just before the layer records), shared by every layer.
struct TrunkGeo {
    int32_t n, h, w, ha, wa, hp, wp, cs16, pad, nbx, nby, ntiles, err, r0, r1, r2;
};

static inline __host__ __device__ size_t trunk_rec_off(int ntiles) {
    return ((size_t)ntiles + 4 + 15) / 16 * 16 + 16;  // words; geometry at rec_off - 16
}

size_t trunk_state_words(int n, int ha, int wa);

typedef const __attribute__((address_space(4))) TrunkRec const_rec;
typedef const __attribute__((address_space(4))) TrunkRec const_rec_t;
typedef const __attribute__((address_space(4))) TrunkGeo const_geo;
__device__ __forceinline__ int rec_xp(const_rec_t& r) { return (int)(r.planes & 0xffff); }
__device__ __forceinline__ int rec_yp(const_rec_t& r) { return (int)(r.planes >> 16); }
__device__ __forceinline__ int rec_r2p(const_rec_t& r) { return (int)(r.shape & 0xffff); }
__device__ __forceinline__ int rec_nch(const_rec_t& r) { return (int)((r.shape >> 16) & 255); }
__device__ __forceinline__ int rec_kind(const_rec_t& r) { return (int)(r.shape >> 24); }
__device__ __forceinline__ int rec_first_new(const_rec_t& r) { return (int)(r.deps & 255); }
__device__ __forceinline__ bool rec_fold(const_rec_t& r) { return ((r.deps >> 8) & 1) != 0; }
__device__ __forceinline__ uint32_t rec_idv(const_rec_t& r) { return r.deps >> 16; }

__device__ __forceinline__ void raw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// Neighbour of tile t polled by this lane (lanes 0..8: the 3x3 neighbourhood), or -1.
__device__ __forceinline__ int nb_of(int t, int nbx, int nby) {
    const int lane = threadIdx.x & 63;
    if (lane >= 9) return -1;
    const int bx = t % nbx, tmp = t / nbx, by = tmp % nby, img = tmp / nby;
    const int yy = by + lane / 3 - 1, xx = bx + lane % 3 - 1;
    return (yy >= 0 && yy < nby && xx >= 0 && xx < nbx) ? (img * nby + yy) * nbx + xx : -1;
}

// s_sleep between two polls of a dependency wait (units of 64 clocks).  A spinning wave's polls
// take issue slots from the wave computing beside it on the same SIMD (the other workgroup of the
// CU) and draw power under the clock cap; A/B builds: _build.build_trunk_alt.
#ifndef ISR_TRUNK_SPIN_SLEEP
#define ISR_TRUNK_SPIN_SLEEP 1
#endif

__device__ __forceinline__ unsigned poll_load(const unsigned* progress, int nb) {
    return __hip_atomic_load(progress + (nb < 0 ? 0 : nb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Blocking wave-level wait for the neighbourhood: every lane leaves with the dependency met or
// the launch given up (bounded spin, then state[1] = gen, and every later wait returns at once
// so the grid always drains; the host reads state[1] == state[0] as "outputs invalid").
__device__ __forceinline__ void dep_wait(unsigned* state, int nb, unsigned need, unsigned gen) {
    const unsigned* progress = state + 4;
    for (unsigned spins = 0;; ++spins) {
        const unsigned v = poll_load(progress, nb);
        if (__all(nb < 0 || (int)(v - need) >= 0)) break;
        if ((spins & 255) == 255 && __hip_atomic_load(state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen)
            break;
        if (spins > (1u << 18)) {
            if ((threadIdx.x & 63) == 0) {
                __hip_atomic_store(state + 1, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(state + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sticky count
            }
            break;
        }
        __builtin_amdgcn_s_sleep(ISR_TRUNK_SPIN_SLEEP);
    }
}

__device__ __forceinline__ void acquire_fence() {
    if ((threadIdx.x & 63) == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Buffer resource over [p, p + bytes): num_records is the tensor's real extent, so an offset past
// it reads zeros / drops the store instead of touching whatever lies beyond the allocation.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_n(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// LDS halo image of one chunk: pixel q = row * 34 + col holds 2 units of 16 B (8 channels);
// unit (q, c) sits at 2q + (c ^ bit 3 of col).  The swizzle depends on the column only, so the
// rows a wave reads at one dx share one per-lane address (row offsets are immediates), and the
// 16 lanes of a ds_read_b128 group (columns 8 apart pair up) still hit 16 distinct bank slots.
template <int HQ>
__device__ __forceinline__ uint32_t halo_piece_off(int j, int lane, int wp) {
    const int u = j * 64 + lane;
    const int q = u >> 1;
    if (q >= HQ) return 0;  // tail of the last piece: never read
    const int row = q / tk::HC, col = q - row * tk::HC;
    const int cc = (u & 1) ^ ((col >> 3) & 1);
    return (uint32_t)((row * wp + col) * 32 + cc * 16);
}

// s_waitcnt vmcnt(n) for a run-time n (0..63): this wave's n youngest vector-memory
// instructions may stay in flight.
__device__ __forceinline__ void wait_vm(uint32_t n) {
#define ISR_VMW(k)                                        \
    case k:                                               \
        asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
        break;
    switch (n) {
        ISR_VMW(1) ISR_VMW(2) ISR_VMW(3) ISR_VMW(4) ISR_VMW(5) ISR_VMW(6) ISR_VMW(7) ISR_VMW(8) ISR_VMW(9)
        ISR_VMW(10) ISR_VMW(11) ISR_VMW(12) ISR_VMW(13) ISR_VMW(14) ISR_VMW(15) ISR_VMW(16) ISR_VMW(17)
        ISR_VMW(18) ISR_VMW(19) ISR_VMW(20) ISR_VMW(21) ISR_VMW(22) ISR_VMW(23) ISR_VMW(24) ISR_VMW(25)
        ISR_VMW(26) ISR_VMW(27) ISR_VMW(28) ISR_VMW(29) ISR_VMW(30) ISR_VMW(31) ISR_VMW(32) ISR_VMW(33)
        ISR_VMW(34) ISR_VMW(35) ISR_VMW(36) ISR_VMW(37) ISR_VMW(38) ISR_VMW(39) ISR_VMW(40) ISR_VMW(41)
        ISR_VMW(42) ISR_VMW(43) ISR_VMW(44) ISR_VMW(45) ISR_VMW(46) ISR_VMW(47) ISR_VMW(48) ISR_VMW(49)
        ISR_VMW(50) ISR_VMW(51) ISR_VMW(52) ISR_VMW(53) ISR_VMW(54) ISR_VMW(55) ISR_VMW(56) ISR_VMW(57)
        ISR_VMW(58) ISR_VMW(59) ISR_VMW(60) ISR_VMW(61) ISR_VMW(62) ISR_VMW(63)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef ISR_VMW
}

template <int V> struct TIC { static constexpr int value = V; };

// A operand of the residual fold: (1/s1) I on couts [16 h16, 16 h16 + 16) of a 32-cout
// fragment (lane l supplies A[l & 31][8 (l >> 5) .. + 8]); conv3x3.hip builds the same.
template <bool FRESH = false>
__device__ __forceinline__ bf16x8 fold_a_bits(uint32_t idv, int h16) {
    int lane = threadIdx.x & 63;
    // FRESH: an opaque copy of the lane id, so the operand is rebuilt at each use (a few VALU ops
    // in the MFMA shadow) instead of being hoisted and kept live in 8 VGPRs across the chunks
    if constexpr (FRESH) asm volatile("" : "+v"(lane));
    const int j = (lane & 31) - 16 * h16 - 8 * (lane >> 5);
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    u32x4 r;
#pragma unroll
    for (int d = 0; d < 4; ++d) r[d] = j == 2 * d ? idv : (j == 2 * d + 1 ? idv << 16 : 0u);
    return __builtin_bit_cast(bf16x8, r);
}


int trunk_prep_launch(const isr_chain_desc* cd, int th, hipStream_t s);

}  // namespace isr
