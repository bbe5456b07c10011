// Elementwise glue on channel-blocked bf16 views (see isr_ew_desc in isr.h).
// One thread per (pixel, 8 channels): 16-byte loads/stores, whole computed
// region (ha x wa), zeros written outside the valid h x w region.
#include "isr_common.h"

namespace isr {

__global__ __launch_bounds__(256) void ew_combine_kernel(isr_ew_desc d) {
    const int cg = d.c / 8;
    const size_t total = (size_t)d.n * d.ha * d.wa * cg;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        // channel group innermost within a 16-channel plane pair, then x, y, plane, image:
        // consecutive threads touch consecutive 16-byte units of one plane row.
        size_t r = i;
        const int half = r % 2; r /= 2;
        const int x = r % d.wa; r /= d.wa;
        const int y = r % d.ha; r /= d.ha;
        const int pl = r % (d.c / 16);
        const int img = (int)(r / (d.c / 16));
        const int c = pl * 16 + half * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y < d.h && x < d.w) {
            float t[8];
            load8_bf16(view_at(d.a, img, y, x, c), t);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = t[k] * d.sa;
            if (d.b.data) {
                load8_bf16(view_at(d.b, img, y, x, c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] += t[k] * d.sb;
            }
            if (d.m.data) {
                load8_bf16(view_at(d.m, img, y, x, c), t);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = t[k] > 0.f ? v[k] : v[k] * d.mslope;
            }
        }
        store8_bf16(view_at(d.y, img, y, x, c), v);
    }
}

int ew_combine_dispatch(const isr_ew_desc* d, hipStream_t s) {
    const size_t total = (size_t)d->n * d->ha * d->wa * (d->c / 8);
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(ew_combine_kernel, dim3(blocks), dim3(256), 0, s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace isr
