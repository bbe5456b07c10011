// Weight / bias gradients of the two 9x9 convs of the generator on MFMA:
//   tail  ConvWithoutBN(64, 3, 9)  (conv2, utils/models.py:607, :636):
//         dW[co][ci][ky][kx] = sum_{y,x} Gp[co][y][x]   * U[ci][y+ky-4][x+kx-4]
//   head  ConvWithoutBN(3, 64, 9)  (conv0, utils/models.py:596, :625):
//         dW[co][ci][ky][kx] = sum_{y,x} Gq[co][y][x]   * X[ci][y+ky-4][x+kx-4]
// where the 3-channel operand ("P": Gp = tail pre-tanh gradient, X = the
// normalised network input) is NCHW fp32 and the 64-channel operand ("Q": U =
// last Scaler output, Gq = head pre-activation gradient) is channel-blocked
// bf16.  Both are written as  sum_{y,x} P[p][y + A(ky-4)][x + S(kx-4)] *
// Q[q][y + B(ky-4)][x]  (tail: A=0, S=-1, B=1 after substituting x → x-kx+4;
// head: A=1, S=+1, B=0).
//
// GEMM: M = (p, kx) = 27 of 32 rows, N = q = 64 (2 fragments), K = pixels; the
// three waves of a block own ky = 3w..3w+2.  The P tile is staged to LDS as bf16
// in 8 copies shifted by one element each, so the 8 consecutive pixels an A
// fragment lane needs at any kx shift are one aligned 16-byte read; the Q tile
// is staged with global_load_lds and read with ds_read_b64_tr_b16 (as in
// wgrad3x3.hip).  Split-K partials + reduce as in wgrad3x3.hip.
#include "isr_common.h"

namespace isr {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_w9;

__device__ __forceinline__ bf16x4 lds_tr4_w9(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_w9*)(p));
}

template <int HEAD_>
struct W9 {
    static constexpr int HEAD = HEAD_;
    static constexpr int A = HEAD ? 1 : 0, S = HEAD ? 1 : -1, B = HEAD ? 0 : 1;
    static constexpr int TY = 4, WM = 3, NT = 192;
    static constexpr int QROWS = TY + 8 * B, PROWS = TY + 8 * A;
    static constexpr int QPL = 4;                           // 64 channels
    static constexpr int Q_PLANE = QROWS * 1024 + 128;      // ≡ 128 (mod 256): tr-read group halves on disjoint banks
    static constexpr int PCOLS = 48;                        // tile cols x0-4 .. x0+35 (+ room for the 8 shifts)
    static constexpr int P_COPY = 4 * PROWS * PCOLS * 2;    // 4 channels (the 4th zero) x rows x cols bf16
    static constexpr int Q_BYTES = QPL * Q_PLANE;
    static constexpr int LDS = Q_BYTES + 8 * P_COPY;
    static constexpr int Q_INSTR = QPL * QROWS;
    static constexpr int IPW = (Q_INSTR + WM - 1) / WM;
    static_assert(LDS <= 163840, "LDS");
};

struct W9Args {
    isr_wgrad9_desc d;
    float* ws;  // [splits][9 ky][32 m][64 q]  then [splits][64] bias partials
    int splits, tiles;
};

template <class C>
__global__ __launch_bounds__(C::NT) void wgrad9x9_kernel(W9Args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const isr_wgrad9_desc& d = a.d;
    const int split = xcd_remap(blockIdx.x, gridDim.x);
    const int t0 = (int)((long)split * a.tiles / a.splits), t1 = (int)((long)(split + 1) * a.tiles / a.splits);
    const int wave = wave_id();
    const int lane = threadIdx.x & 63, l31 = lane & 31, hh = lane >> 5;
    const int nbx = d.wa / 32, nby = d.ha / C::TY;
    const size_t qps = plane_bytes(d.q);
    const int qrow = d.q.wp * 32;
    const size_t pplane = (size_t)d.h * d.w;
    const float* P = d.p;
    char* pl = smem + C::Q_BYTES;

    f32x16 acc[3][2];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[k][f][g] = 0.f;
    float bq[2] = {0.f, 0.f};   // head: sum of Q (bias of the 64-channel conv), wave 0
    float bp[3] = {0.f, 0.f, 0.f};  // tail: sum of P over interior pixels (bias of the 3-channel conv)

    // A-fragment lane geometry: m = l31 = (p, kx)
    const int mp = l31 < 27 ? l31 / 9 : 3, mkx = l31 < 27 ? l31 % 9 : 0;
    // tr-read lane geometry (see wgrad3x3.hip)
    const int gi = (lane >> 4) & 1, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int b_lane = gi * C::Q_PLANE + (8 * hh + q4) * 32 + 8 * p4;

    for (int t = t0; t < t1; ++t) {
        const int bx = t % nbx;
        int r_ = t / nbx;
        const int by = r_ % nby, img = r_ / nby;
        const int x0 = bx * 32, y0 = by * C::TY;
        __syncthreads();  // previous tile's reads done
        // ---- Q rows y0 - 4B .. via glds (one row of one plane per instruction)
        {
            const char* qb = view_at(d.q, img, y0 - 4 * C::B, x0, 0);
#pragma unroll
            for (int k = 0; k < C::IPW; ++k) {
                const int j = wave + C::WM * k;
                if (j < C::Q_INSTR) {
                    const int plq = j / C::QROWS, rr = j - plq * C::QROWS;
                    glds16(qb + plq * qps + (size_t)rr * qrow + lane * 16, smem + plq * C::Q_PLANE + rr * 1024);
                }
            }
        }
        // ---- P rows y0 - 4A .., cols x0-4 .. x0+35 → bf16, 8 shifted copies
        for (int e = threadIdx.x; e < 4 * C::PROWS * 40; e += C::NT) {
            const int c = e / (C::PROWS * 40);
            const int rem = e - c * (C::PROWS * 40);
            const int row = rem / 40, col = rem - row * 40;
            const int yy = y0 - 4 * C::A + row, xx = x0 - 4 + col;
            float v = 0.f;
            if (c < 3 && yy >= 0 && yy < d.h && xx >= 0 && xx < d.w) {
                v = P[(size_t)(img * 3 + c) * pplane + (size_t)yy * d.w + xx];
                if (!C::HEAD && col >= 4 && col < 36) bp[c] += v;
            }
            const __bf16 bv = (__bf16)v;
            __bf16* base = reinterpret_cast<__bf16*>(pl) + (c * C::PROWS + row) * C::PCOLS + col;
#pragma unroll
            for (int j = 0; j < 8; ++j) base[j * (C::P_COPY / 2) + j] = bv;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();

#pragma unroll
        for (int kg = 0; kg < 2 * C::TY; ++kg) {
            const int r = kg >> 1, c0 = (kg & 1) * 16;
            // B fragments (Q), per ky when B=1 (tail), shared when B=0 (head)
            bf16x8 fb[3][2];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int ky = 3 * wave + k;
                const int qr = r + C::B * ky;  // Q tile row (tile rows start at y0 - 4B)
#pragma unroll
                for (int f = 0; f < 2; ++f) {
                    if (C::B == 0 && k > 0) {
                        fb[k][f] = fb[0][f];
                    } else {
                        const char* pb = smem + b_lane + 2 * f * C::Q_PLANE + (qr * 32 + c0) * 32;
                        bf16x4 lo = lds_tr4_w9(pb), hi = lds_tr4_w9(pb + 4 * 32);
                        fb[k][f] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    }
                }
            }
            if (C::HEAD && wave == 0) {
#pragma unroll
                for (int f = 0; f < 2; ++f)
#pragma unroll
                    for (int e = 0; e < 8; ++e) bq[f] += (float)fb[0][f][e];
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int ky = 3 * wave + k;
                // A fragment: P[mp][row][col .. col+7], col = c0 + 8h + S(kx-4) + 4 (tile col index)
                const int prow = r + C::A * ky;
                const int col = c0 + 8 * hh + C::S * (mkx - 4) + 4;
                const int j = (8 - (col & 7)) & 7;
                const bf16x8 fa = *reinterpret_cast<const bf16x8*>(
                    pl + j * C::P_COPY + (((mp * C::PROWS + prow) * C::PCOLS) + col + j) * 2);
#pragma unroll
                for (int f = 0; f < 2; ++f) acc[k][f] = mfma32(fa, fb[k][f], acc[k][f]);
            }
        }
    }

    // ---- partials: D[m = (g&3)+8(g>>2)+4h][q = f*32 + l31]
    float* wsp = a.ws + (size_t)split * 9 * 32 * 64;
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int m = (g & 3) + 8 * (g >> 2) + 4 * hh;
                wsp[((3 * wave + k) * 32 + m) * 64 + f * 32 + l31] = acc[k][f][g];
            }
    float* bsp = a.ws + (size_t)a.splits * 9 * 32 * 64 + (size_t)split * 64;
    if (C::HEAD) {
        if (wave == 0) {
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const float v = bq[f] + __shfl_xor(bq[f], 32);
                if (hh == 0) bsp[f * 32 + gi * 16 + (lane & 15)] = v;
            }
        }
    } else {
        // block reduction of the 3 P sums through LDS (after everyone is done with the tile)
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = bp[c];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0) red[wave * 4 + c] = v;
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            bsp[threadIdx.x] = red[threadIdx.x] + red[4 + threadIdx.x] + red[8 + threadIdx.x];
        }
    }
}

// dW in the reference OIHW layout: tail [3][64][9][9] (co = p, ci = q), head [64][3][9][9] (co = q, ci = p)
__global__ __launch_bounds__(256) void wgrad9_reduce_kernel(W9Args a) {
    // A block owns 64 consecutive entries of the partial-sum layout
    // [split][ky][r = p*9 + kx (32)][q (64)] (+ the bias partials after it); its 4 waves
    // take every 4th split, each wave reading 64 consecutive floats (256 B) per split,
    // and the 4 shares meet in LDS.  The OIHW output is written scattered, once.
    __shared__ float red[4][64];
    const isr_wgrad9_desc& d = a.d;
    const int per = 9 * 32 * 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int o = blockIdx.x * 64 + lane;
    const bool bias = o >= per;
    const int c = o - per;
    float s = 0.f;
    if (!bias || (d.db && c < 64)) {
        const float* src = bias ? a.ws + (size_t)a.splits * per + c : a.ws + o;
        const size_t stride = bias ? 64 : per;
        for (int sp = wave; sp < a.splits; sp += 4) s += src[(size_t)sp * stride];
    }
    red[wave][lane] = s;
    __syncthreads();
    if (wave != 0) return;
    s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (!bias) {
        const int q = o & 63, r = (o >> 6) & 31, ky = o >> 11;
        if (r >= 27) return;
        const int p = r / 9, kx = r - 9 * (r / 9);
        const int idx = d.head ? ((q * 3 + p) * 9 + ky) * 9 + kx   // dw [64][3][9][9]
                               : ((p * 64 + q) * 9 + ky) * 9 + kx; // dw [3][64][9][9]
        d.dw[idx] = s * d.scale;
    } else if (d.db && c < (d.head ? 64 : 3)) {
        d.db[c] = s * d.scale;
    }
}

template <class C>
static void w9_geometry(const isr_wgrad9_desc* d, int* tiles, int* splits) {
    *tiles = d->n * (d->ha / C::TY) * (d->wa / 32);
    int s = d->splits > 0 ? d->splits : 512;
    *splits = s < *tiles ? s : *tiles;
}

template <class C>
static int launch_w9(const isr_wgrad9_desc* d, void* ws, size_t ws_bytes, hipStream_t s) {
    W9Args a;
    a.d = *d;
    w9_geometry<C>(d, &a.tiles, &a.splits);
    if (ws_bytes < (size_t)a.splits * (9 * 32 * 64 + 64) * 4) return -3;
    a.ws = (float*)ws;
    auto kern = wgrad9x9_kernel<C>;
    lds_limit((const void*)kern, C::LDS);
    hipLaunchKernelGGL(kern, dim3(a.splits), dim3(C::NT), C::LDS, s, a);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(wgrad9_reduce_kernel, dim3((9 * 32 * 64 + 64) / 64), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t wgrad9x9_workspace_bytes(const isr_wgrad9_desc* d) {
    int tiles, splits;
    if (d->head) w9_geometry<W9<1>>(d, &tiles, &splits);
    else w9_geometry<W9<0>>(d, &tiles, &splits);
    return (size_t)splits * (9 * 32 * 64 + 64) * 4;
}

int wgrad9x9_dispatch(const isr_wgrad9_desc* d, void* ws, size_t ws_bytes, hipStream_t s) {
    return d->head ? launch_w9<W9<1>>(d, ws, ws_bytes, s) : launch_w9<W9<0>>(d, ws, ws_bytes, s);
}

}  // namespace isr
