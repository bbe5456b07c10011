// 3x3 stride-1 'same' convolution as an implicit GEMM on CDNA4 MFMA
// (v_mfma_f32_32x32x16_bf16), NHWC bf16 activations, fp32 accumulation.
//
// Replaces the ATen convolution behind Conv / ConvWithoutBN / RDB / RRDB /
// Scaler of the reference (utils/models.py:75-111, 174-199, 245-271, 298-317,
// 572-589) together with their BN (folded), LeakyReLU, torch.cat, residual
// add/mul and PixelShuffle, which all become the epilogue of one launch.
//
// Block tile: TH = R*WM output rows x 32 output columns x CT = NF*32 output
// channels.  Wave w owns rows [w*R, w*R+R).  GEMM view per block:
//   M = 32 pixels of one row (one MFMA row-fragment per output row),
//   N = CT output channels (NF fragments of 32),
//   K = 9 taps x Cin, walked in chunks of 32 input channels.
// Per chunk the (TH+2) x 34 x 32ch halo image and the chunk's packed weights
// are copied global → LDS with global_load_lds_dwordx4 (double-buffered), then
// each wave walks (dx, k-step) and re-uses every A fragment (one input row)
// for the up-to-3 output rows (dy taps) that read it: R+2 A reads feed 3*R*NF
// MFMAs.  The epilogue transposes the accumulators through LDS so that every
// lane stores 16 contiguous bytes (8 channels) of one pixel.
#include "isr_common.h"

namespace isr {

template <int R, int WM, int NF>
struct C3 {
    static constexpr int TH = R * WM;
    static constexpr int TW = 32;
    static constexpr int HR = TH + 2;  // halo rows
    static constexpr int HC = TW + 2;  // halo cols
    static constexpr int CT = NF * 32; // output channels per block
    static constexpr int KC = 32;      // input channels per chunk
    static constexpr int HALO_UNITS = HR * HC * 4;
    static constexpr int HALO_INSTR = (HALO_UNITS + 63) / 64;
    static constexpr int HALO_BYTES = HALO_INSTR * 1024;
    static constexpr int W_UNITS = 9 * 2 * CT * 2; // [tap][ks][n][hpos] x 16 B
    static constexpr int W_INSTR = W_UNITS / 64;
    static constexpr int W_BYTES = W_UNITS * 16;
    static constexpr int STAGE = HALO_BYTES + W_BYTES;
    static constexpr int NT = 64 * WM;
    static constexpr int INSTR = HALO_INSTR + W_INSTR;
    static constexpr int IPW = (INSTR + WM - 1) / WM; // glds instructions per wave per chunk
    static constexpr int EPS = CT + 4;                // floats per pixel in the epilogue image
    static constexpr int EP_BYTES = WM * R * 32 * EPS * 4;
    static constexpr int LDS = (2 * STAGE > EP_BYTES) ? 2 * STAGE : EP_BYTES;
    static_assert(W_UNITS % 64 == 0, "weight stage must be whole glds instructions");
    static_assert(LDS <= 163840, "LDS budget");
};

// Packed weight layout for cout tile `ct`, input chunk `ch`:
//   [tap 9][ks 2][n CT][hpos 2][8 bf16]  (one contiguous W_BYTES block)
// element (tap=dy*3+dx, ks, n, hpos, e) = W[ct*CT+n][ch*32 + ks*16 + h*8 + e][dy][dx],
// h = hpos ^ ((n >> 3) & 1) (bank swizzle of the B-fragment ds_read_b128).
__device__ __forceinline__ int wunit(int tap, int ks, int n, int h, int CT) {
    return ((tap * 2 + ks) * CT + n) * 2 + (h ^ ((n >> 3) & 1));
}

template <int R, int WM, int NF>
__global__ __launch_bounds__(64 * WM) void conv3x3_fwd_kernel(isr_conv_desc d) {
    using C = C3<R, WM, NF>;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int nct = d.cout / C::CT;
    const int img = blockIdx.z / nct;
    const int ct = blockIdx.z - img * nct;
    const int x0 = blockIdx.x * C::TW;
    const int y0 = blockIdx.y * C::TH;
    const int wave = wave_id();
    const int lane = threadIdx.x & 63;
    const int l31 = lane & 31;
    const int hh = lane >> 5;
    const int nchunks = d.cin / C::KC;

    // ---- per-lane glds source offsets (chunk-invariant) -------------------
    const char* xbase = view_px(d.x, img, y0 - 1, x0 - 1);
    const char* wbase = (const char*)d.wpack + (size_t)ct * nchunks * C::W_BYTES;
    const int xrow_bytes = d.x.wp * d.x.cs * 2;
    const int xpix_bytes = d.x.cs * 2;
    uint32_t off[C::IPW];
#pragma unroll
    for (int k = 0; k < C::IPW; ++k) {
        const int j = wave + WM * k;
        uint32_t o = 0;
        if (j < C::HALO_INSTR) {
            const int u = j * 64 + lane;
            if (u < C::HALO_UNITS) {
                const int q = u >> 2;
                const int cpos = u & 3;
                const int row = q / C::HC;
                const int col = q - row * C::HC;
                const int c = cpos ^ ((q >> 2) & 3);
                o = (uint32_t)(row * xrow_bytes + col * xpix_bytes + c * 16);
            }
        } else {
            o = (uint32_t)((j - C::HALO_INSTR) * 1024 + lane * 16);
        }
        off[k] = o;
    }

    auto stage = [&](int chunk, int buf) {
        char* dst = smem + buf * C::STAGE;
        const char* xs = xbase + chunk * (C::KC * 2);
        const char* ws = wbase + (size_t)chunk * C::W_BYTES;
#pragma unroll
        for (int k = 0; k < C::IPW; ++k) {
            const int j = wave + WM * k;
            if (j < C::INSTR) {
                const char* src = (j < C::HALO_INSTR ? xs : ws) + off[k];
                glds16(src, dst + j * 1024);
            }
        }
    };

    f32x16 acc[R][NF];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[r][f][g] = 0.f;

    stage(0, 0);
    wait_vm0();
    __syncthreads();

    const int qw = wave * R * C::HC + l31; // halo pixel of (row w*R, col l31)
    for (int chunk = 0; chunk < nchunks; ++chunk) {
        const int buf = chunk & 1;
        if (chunk + 1 < nchunks) stage(chunk + 1, buf ^ 1);
        const char* hs = smem + buf * C::STAGE;
        const char* ws = hs + C::HALO_BYTES;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 b[3][NF];
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int f = 0; f < NF; ++f)
                        b[dy][f] = lds_read16(ws + wunit(dy * 3 + dx, ks, f * 32 + l31, hh, C::CT) * 16);
                const int c = 2 * ks + hh;
#pragma unroll
                for (int i = 0; i < R + 2; ++i) {
                    const int q = qw + i * C::HC + dx;
                    const bf16x8 a = lds_read16(hs + halo_unit(q, c) * 16);
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
        wait_vm0();
        __syncthreads();
    }

    // ---- epilogue: accumulators → LDS [row][px][CT] fp32 → 8-channel stores
    float* ep = reinterpret_cast<float*>(smem) + wave * (R * 32 * C::EPS);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int px = (g & 3) + 8 * (g >> 2) + 4 * hh;
                ep[(r * 32 + px) * C::EPS + f * 32 + l31] = acc[r][f][g];
            }
    __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();

    Epi e;
    e.bias = d.bias; e.slope = d.slope; e.s1 = d.s1; e.s2 = d.s2;
    e.y = d.y; e.y2 = d.y2; e.r1 = d.r1; e.r2 = d.r2; e.h = d.h; e.w = d.w;
    constexpr int ITEMS = R * C::CT / 16; // per lane
    if (d.shuffle == 2) {
        // item → (row r, sub-row i, output col xo in [0,64), 8-channel group cg)
        constexpr int CG = C::CT / 32;
#pragma unroll 4
        for (int it = 0; it < ITEMS; ++it) {
            const int jj = lane + 64 * it;
            const int cg = jj % CG;
            const int rem = jj / CG;
            const int xo = rem & 63;
            const int si = (rem >> 6) & 1;
            const int r = rem >> 7;
            const int xc = xo >> 1, sj = xo & 1;
            const int yy = y0 + wave * R + r;
            const int xx = x0 + xc;
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int col = 4 * (cg * 8 + k) + 2 * si + sj;
                v[k] = ep[(r * 32 + xc) * C::EPS + col] + (e.bias ? e.bias[ct * C::CT + col] : 0.f);
                v[k] = v[k] >= 0.f ? v[k] : v[k] * e.slope;
            }
            if (!(yy < e.h && xx < e.w)) {
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = 0.f;
            }
            char* dst = view_px(e.y, img, 2 * yy + si, 2 * x0 + xo) + (ct * (C::CT / 4) + cg * 8) * 2;
            store8_bf16(dst, v);
        }
    } else {
        constexpr int CG = C::CT / 8;
#pragma unroll 4
        for (int it = 0; it < ITEMS; ++it) {
            const int jj = lane + 64 * it;
            const int cg = jj % CG;
            const int p = jj / CG;
            const int r = p >> 5, px = p & 31;
            float v[8];
            const float* src = ep + (r * 32 + px) * C::EPS + cg * 8;
            f32x4 a0 = *reinterpret_cast<const f32x4*>(src);
            f32x4 a1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) { v[k] = a0[k]; v[4 + k] = a1[k]; }
            epi_plain8(e, v, img, y0 + wave * R + r, x0 + px, ct * C::CT + cg * 8);
        }
    }
}

template <int R, int WM, int NF>
static int launch3x3(const isr_conv_desc* d, hipStream_t s) {
    using C = C3<R, WM, NF>;
    auto kern = conv3x3_fwd_kernel<R, WM, NF>;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
        attr = true;
    }
    dim3 grid(d->wa / C::TW, d->ha / C::TH, d->n * (d->cout / C::CT));
    hipLaunchKernelGGL(kern, grid, dim3(C::NT), C::LDS, s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int conv3x3_fwd_dispatch(const isr_conv_desc* d, hipStream_t s) {
    if (d->cout == 32) return launch3x3<4, 4, 1>(d, s);
    return launch3x3<4, 4, 2>(d, s);
}

int conv3x3_cout_tile(int cout) { return cout == 32 ? 32 : 64; }

// ---- weight packing: fp32 OIHW → bf16 [ct][chunk][tap][ks][n][hpos][8] ----
__global__ void pack3x3_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int cout, int cin, int CT) {
    const int nchunks = cin / 32;
    const size_t per_block = (size_t)9 * 2 * CT * 16;
    const size_t total = per_block * nchunks * (cout / CT);
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
        size_t rem = idx;
        const int e = rem % 8; rem /= 8;
        const int hpos = rem % 2; rem /= 2;
        const int n = rem % CT; rem /= CT;
        const int ks = rem % 2; rem /= 2;
        const int tap = rem % 9; rem /= 9;
        const int ch = rem % nchunks; rem /= nchunks;
        const int ct = (int)rem;
        const int h = hpos ^ ((n >> 3) & 1);
        const int co = ct * CT + n;
        const int ci = ch * 32 + ks * 16 + h * 8 + e;
        const int dy = tap / 3, dx = tap % 3;
        out[idx] = (__bf16)w[((size_t)co * cin + ci) * 9 + dy * 3 + dx];
    }
}

size_t conv3x3_packed_bytes(int cout, int cin) { return (size_t)cout * cin * 9 * 2; }

int conv3x3_pack(const float* w, void* out, int cout, int cin, hipStream_t s) {
    const int CT = conv3x3_cout_tile(cout);
    const size_t total = conv3x3_packed_bytes(cout, cin) / 2;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(pack3x3_kernel, dim3(blocks), dim3(256), 0, s, w, (__bf16*)out, cout, cin, CT);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr
