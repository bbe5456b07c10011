/*
 * isr.h — C-ABI of libisr.so, the MI355X (gfx950) kernels behind the
 * image_super_resolution_amd drop-in.
 *
 * The reference (thnak/image_super_resolution) has no FFI/plugin layer: its hot
 * path is torch.nn modules dispatching to ATen convolutions.  Each entry point
 * below replaces one group of those module forwards (cited per function,
 * paths relative to the reference root).  A host binds these with ctypes (see
 * INTEGRATION.md); no torch types cross this boundary.
 *
 * Conventions
 *  - Activations are channel-blocked 2-byte floats ("NC16HW16c": bf16, or fp16 on the
 *    forward descriptors with f16 = 1, the inference default since round 6) in caller-owned device
 *    buffers laid out as [N][cs/16][hp][wp][16] with a zero border of `pad`
 *    pixels on every side: each 16-channel block is a contiguous plane, so a
 *    K-chunk of a convolution reads whole cache lines.  The caller zero-fills a
 *    buffer once; kernels never write the border and write exact zeros at
 *    computed positions outside the valid h x w region, so the border /
 *    alignment slack always reads as the conv's zero padding.
 *  - Computed regions are tile-aligned: ha % ISR_TILE_H == 0, wa % ISR_TILE_W == 0.
 *  - The library never allocates, frees or synchronises; every call takes an
 *    explicit stream and is hipGraph-capturable.
 *  - Return 0 on success, a negative ISR_ERR_* otherwise; isr_last_error()
 *    returns a thread-local message for the last failure.
 */
#ifndef ISR_H
#define ISR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* isr_stream_t; /* == hipStream_t */

#define ISR_OK 0
#define ISR_ERR_BAD_DESC (-1)
#define ISR_ERR_UNSUPPORTED (-2)
#define ISR_ERR_LAUNCH (-3)

#define ISR_TILE_H 32
#define ISR_TILE_W 32

/* A channel slice [coff, coff + k) of a channel-blocked bf16 / fp16 buffer
 * [N][cs/16][hp][wp][16] with border `pad` (cs, coff multiples of 16).
 * Interior pixel (n, y, x), view channel c (ch = coff + c) lives at
 *   data + ((((n*(cs/16) + ch/16)*hp + y + pad)*wp + x + pad)*16 + ch%16) * 2 bytes. */
typedef struct isr_view {
    void* data;
    int32_t hp, wp, cs, pad, coff;
} isr_view;

/* 3x3 stride-1 'same' convolution with fused epilogue:
 *   v = act(conv(x, W) + bias);  v = v*s1 + r1 (if r1);  v = v*s2 + r2 (if r2)
 *   store v to y (PixelShuffle(2)-permuted when shuffle == 2) and to y2 (if set).
 * act is LeakyReLU(slope) (slope = 1 → identity, 0 → ReLU).
 * Replaces: Conv._forward_impl (utils/models.py:97-98, BN folded by
 * fuse_conv_and_bn :366-406), ConvWithoutBN._forward_impl (:195-196),
 * the torch.cat chain + residual of RDB.forward (:265-271; the caller points
 * y at a channel slice of the dense-block buffer), RRDB.forward (:316-317, as
 * r2), ResNet/EResNet trunk add (:615, :647) and Scaler (:572-589: conv →
 * PixelShuffle(2) → LeakyReLU via shuffle == 2). */
typedef struct isr_conv_desc {
    int32_t n, h, w;   /* batch; valid conv height/width (input == output size) */
    int32_t ha, wa;    /* computed (tile-aligned) extent; ha % 32 == 0, wa % 32 == 0 */
    int32_t cin, cout; /* cin % 16 == 0; cout % 32 == 0 (cout % 64 != 0 runs 32-cout tiles) */
    isr_view x;        /* input (cin channels from x.coff) */
    isr_view y;        /* output; for shuffle == 2 its grid is (2h, 2w), cout/4 channels */
    isr_view y2;       /* optional duplicate output (y2.data == NULL → none) */
    isr_view r1, r2;   /* optional residuals (data == NULL → none), cout channels */
    const void* wpack; /* from isr_pack_conv3x3 */
    const float* bias; /* [cout] fp32 or NULL */
    float slope, s1, s2; /* s2 multiplies after r1 even without r2: set 1.0 when unused */
    int32_t shuffle;   /* 1 = plain store, 2 = PixelShuffle(2) store */
    /* Backward-pass extensions (all zero in the forward).  The epilogue order is
     * v = act(acc + bias); v = v*s1 + r1; v = v*s2 + r2; v *= mask; store.
     * Used by the generator backward (utils/models.py forward graph, autograd
     * of train.py:57 / :102): input-gradient convs accumulate into the dense-block
     * gradient buffer and apply LeakyReLU' of the forward activation. */
    isr_view m;        /* optional mask source (data == NULL → none), same grid as y */
    float mslope;      /* output channel c >= m_c0 is multiplied by (m[c] > 0 ? 1 : mslope); with shuffle == 2
                          m is on the shuffled grid and masks every channel (m_c0 = 0) */
    int32_t m_c0;      /* first masked output channel, multiple of 32 */
    int32_t r1_cn;     /* r1 is added only to output channels < r1_cn (0 → all); multiple of 32 */
    int32_t x_sub2;    /* 1: input channel c' = s*(cin/4) + c reads x at pixel (2y + (s>>1), 2x + (s&1)),
                          channel c (x is on the 2h x 2w grid, pad >= 2): the transpose of
                          PixelShuffle(2) (utils/models.py:583) folded into the load; cin % 128 == 0 */
    int32_t taps;      /* 0: all 3x3 taps; 1: only taps {0,1}^2; 2: only taps {1,2}^2 (cout % 64 == 0).
                          A stride-2 3x3 conv (Discriminator, utils/models.py:533-542) is taps=1 over the
                          x_sub2 view with 4*cin phase-expanded weights; its input gradient is taps=2
                          over the output gradient with shuffle == 2 (4*cin phase outputs). */
    int32_t f16;       /* 0: activations (x, y, y2, r1, r2) and wpack are bf16; 1: fp16 (the inference
                          path: 10 mantissa bits instead of 7, the storage type of the reference's own
                          fp16 autocast, train.py:54 / rs.py), wpack from isr_pack_conv3x3_f16.  fp16 is
                          forward-only: m.data == NULL, x_sub2 == 0, taps == 0. */
} isr_conv_desc;

/* 9x9 head conv, 3 → cout (=64) channels, input NCHW (fp32 already normalised,
 * or uint8 with Normalize fused), + bias + LeakyReLU(slope), NHWC bf16 out.
 * Replaces: ResNet.conv0 / EResNet.conv0 (utils/models.py:596, :625) and the
 * Normalize of Model.init_normalize (:731-732; utils/datasets.py:65-71). */
typedef struct isr_head_desc {
    int32_t n, h, w, ha, wa;
    int32_t cout;          /* 64 */
    const void* x;         /* NCHW [n][3][h][w] */
    int32_t x_u8;          /* 0: fp32 input used as is; 1: uint8, (v/255 - mean)/std fused */
    float mean[3], inv_std[3];
    isr_view y, y2;
    const void* wpack;     /* from isr_pack_head9x9 */
    const float* bias;     /* [cout] or NULL */
    float slope;
    /* backward use (zero in the forward): with fp32 input, mean 0, inv_std 1,
     * slope 1 and 180°-rotated, transposed weights this is the input gradient of
     * the 9x9 tail conv (utils/models.py:607, :636); m masks it with
     * LeakyReLU'(m) of slope mslope (the last Scaler's activation). */
    isr_view m;
    float mslope;
    int32_t f16;           /* 1: y / y2 fp16 and wpack from isr_pack_head9x9_f16 (forward only, m.data == NULL) */
} isr_head_desc;

/* 9x9 tail conv, cin (=64) → 3 channels, + bias + tanh, NCHW out (fp32, or
 * uint8 with TanhToArrayImage fused: round_half_even((t+1)/2*255)).
 * Replaces: ResNet.conv2 / EResNet.conv2 (utils/models.py:607, :636) and
 * TanhToArrayImage.forward (:448-451). */
typedef struct isr_tail_desc {
    int32_t n, h, w, ha, wa; /* valid / computed extent of the tail (= output size) */
    int32_t cin;             /* 64 */
    isr_view x;              /* NHWC bf16, pad >= 4 */
    const void* wpack;       /* from isr_pack_tail9x9 */
    const float* bias;       /* [3] or NULL */
    void* y;                 /* NCHW [n][3][h][w] */
    int32_t y_u8;            /* 0: fp32 tanh output; 1: uint8 image */
    int32_t f16;             /* 1: x fp16 and wpack from isr_pack_tail9x9_f16 */
} isr_tail_desc;

/* Weight / bias gradient of a 3x3 'same' conv (the bwd-weight half of autograd
 * through Conv / ConvWithoutBN / RDB / Scaler, utils/models.py:75-111, 174-199,
 * 245-271, 572-589, driven by train.py:57 / :102):
 *   dw[co][ci][ky][kx] = scale * sum_{n,y,x} g[n][co][y][x] * x[n][ci][y+ky-1][x+kx-1]
 *   db[co]             = scale * sum_{n,y,x} g[n][co][y][x]
 * g must be zero outside the valid h x w region (every isr kernel writes zeros there).
 * Needs a caller-owned workspace of isr_wgrad3x3_workspace_bytes(desc) bytes
 * (split-K partial sums); dw / db are overwritten. */
typedef struct isr_wgrad_desc {
    int32_t n, h, w, ha, wa; /* conv output grid (= input grid) */
    int32_t cin, cout;       /* multiples of 32 */
    isr_view x;              /* forward input, cin channels, pad >= 1 */
    isr_view g;              /* gradient w.r.t. the conv output, cout channels */
    int32_t g_sub2;          /* 1: g is the PixelShuffle(2)'d gradient on the 2h x 2w grid with cout/4
                                channels (Scaler, utils/models.py:583); cout % 128 == 0 */
    float scale;
    float* dw;               /* [cout][cin][3][3] fp32 */
    float* db;               /* [cout] fp32 or NULL */
    int32_t splits;          /* split-K count; 0 = library choice */
    int32_t x_sub2;          /* 1: x is read as PixelShuffle(2)^T of a 2h x 2w buffer (pad >= 2): kernel input
                                channel s*(cin/4) + c = x[c] at (2y + (s>>1), 2x + (s&1)); cin % 128 == 0.
                                With taps == 1 this is the weight gradient of a stride-2 conv (Discriminator,
                                utils/models.py:533-542) on its phase decomposition. */
    int32_t taps;            /* 0: all 3x3 taps; 1: only taps {0,1}^2 (dw at other taps left undefined) */
} isr_wgrad_desc;

/* Weight / bias gradients of the 9x9 convs (same workspace contract):
 *   head = 1: conv0 3 → 64 (utils/models.py:596, :625): p = the (normalised)
 *             network input, q = gradient wrt conv0's pre-activation output;
 *             dw [64][3][9][9], db [64].
 *   head = 0: conv2 64 → 3 (utils/models.py:607, :636): p = gradient wrt
 *             conv2's pre-tanh output, q = conv2's input (pad >= 4);
 *             dw [3][64][9][9], db [3].
 * dw[co][ci][ky][kx] = scale * sum_{n,y,x} gout[co][y][x] * in[ci][y+ky-4][x+kx-4]. */
typedef struct isr_wgrad9_desc {
    int32_t n, h, w, ha, wa;
    int32_t head;
    const float* p;          /* NCHW fp32 [n][3][h][w] */
    isr_view q;              /* 64 channels, zero outside h x w */
    float scale;
    float* dw;
    float* db;               /* or NULL */
    int32_t splits;          /* 0 = library choice */
} isr_wgrad9_desc;

size_t isr_wgrad9x9_workspace_bytes(const isr_wgrad9_desc* d);
int isr_wgrad9x9(const isr_wgrad9_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s);

size_t isr_wgrad3x3_workspace_bytes(const isr_wgrad_desc* d);
int isr_wgrad3x3(const isr_wgrad_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s);
/* isr_wgrad3x3 in two launches: the split-K partial sums into `workspace`, then their reduction
 * into dw / db (same descriptor and workspace; the caller orders the second after the first, on
 * another stream too, and keeps the workspace untouched in between).  Lets a caller take the
 * reductions off the stream that chains the weight-gradient kernels (train_engine.py). */
/* Up to 5 weight gradients over one pixel grid in one launch (plus one reduce launch): the 5 convs
 * of an RDB (utils/models.py:265-271) read one dense buffer and one gradient buffer; their (co, ci)
 * tile pairs share one grid, so ~5x fewer split-K partials fill the chip.  Members: plain 3x3
 * (g_sub2 = x_sub2 = taps = 0), cin / cout multiples of 32, the same n / ha / wa; `splits` is
 * ignored.  Each member's dw / db / scale as in isr_wgrad3x3; one workspace of
 * isr_wgrad3x3_group_workspace_bytes(descs, n) bytes. */
size_t isr_wgrad3x3_group_workspace_bytes(const isr_wgrad_desc* descs, int32_t n);
int isr_wgrad3x3_group(const isr_wgrad_desc* descs, int32_t n, void* workspace, size_t ws_bytes, isr_stream_t s);
/* The grouped launch by an explicit form: 0 = production (isr_wgrad3x3_group: asm transposing
 * LDS reads with counted waits), 1 = the same tiles and splits with compiler-visible LDS reads
 * (the bit-identical reference the production form is tested against); same workspace size. */
int isr_wgrad3x3_group_variant(const isr_wgrad_desc* descs, int32_t n, int32_t variant, void* workspace,
                               size_t ws_bytes, isr_stream_t s);
int isr_wgrad3x3_partials(const isr_wgrad_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s);
int isr_wgrad3x3_reduce(const isr_wgrad_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s);
/* The same computation by an explicit kernel variant, with its own workspace size: 0 = production
 * (isr_wgrad3x3), 16 = the production tiles and split counts with compiler-visible LDS reads (the
 * bit-identical reference of the asm-read forms); 1..15 = earlier tile forms, in tuning builds only
 * (-DISR_TUNING; a production library returns ISR_ERR_UNSUPPORTED / 0 bytes for them). */
size_t isr_wgrad3x3_variant_workspace_bytes(const isr_wgrad_desc* d, int32_t variant);
int isr_wgrad3x3_variant(const isr_wgrad_desc* d, int32_t variant, void* workspace, size_t ws_bytes, isr_stream_t s);

/* Elementwise combine on channel-blocked views (backward glue):
 *   y = (a*sa + b*sb) * (m > 0 ? 1 : mslope)   over c channels; b, m optional;
 * y is zero outside the valid h x w region.  Replaces the autograd sum at the
 * generator trunk (utils/models.py:615, :647: inputs + conv1(residual(inputs)))
 * and conv0's LeakyReLU backward. */
typedef struct isr_ew_desc {
    int32_t n, h, w, ha, wa, c;
    isr_view y, a, b, m;
    float sa, sb, mslope;
} isr_ew_desc;
int isr_ew_combine(const isr_ew_desc* d, isr_stream_t s);

/* PixelShuffle(2) + LeakyReLU(mslope) between channel-blocked views (same descriptor):
 *   y[c] at (y, x) = act(sa * a[4c + 2*(y%2) + (x%2)] at (y/2, x/2)),  c < d->c
 * (n, h, w, ha, wa) is the OUTPUT grid (even); a holds 4c channels on the
 * (h/2) x (w/2) grid; b and m must be NULL.  Zeros outside the valid region.
 * Replaces: Denoise.residual_conv1 = Sequential(PixelShuffle(2), LeakyReLU(0.2))
 * (utils/models.py:687) applied to the output of a ResidualBlock1 (:202-209),
 * whose residual add precedes the shuffle so it cannot ride a conv epilogue. */
int isr_pixel_shuffle2(const isr_ew_desc* d, isr_stream_t s);
/* Its transpose, the PixelShuffle(2) input gradient (Denoise training, train.py:204-205):
 *   y[4c + s] at (y, x) = sa * a[c] at (2y + s/2, 2x + s%2) * (m there > 0 ? 1 : mslope)
 * (n, h, w, ha, wa) is the OUTPUT (half-resolution) grid, d->c its channel count
 * (multiple of 64); a and the optional LeakyReLU' mask source m hold c/4 channels on
 * the 2h x 2w grid (rows / cols up to 2ha / 2wa are read); b must be NULL. */
int isr_pixel_unshuffle2(const isr_ew_desc* d, isr_stream_t s);

/* Training-data transform of SR_dataset (utils/datasets.py:344-355) over a batch of uint8 HR
 * crops in ONE launch: lr = Normalize(cv2 INTER_LINEAR uint8 resize by `scale`, :302-304: at the
 * integer factors the block's centre pixel (odd) or its centre 2x2 mean rounded half up (even)),
 * hr = 2x/255 - 1 (PIL_to_tanh, :96-106) or Normalize(x) when hr_norm (SRGAN mode, :336-339).
 * crops [n][3][t][t] uint8, hr [n][3][t][t] fp32, lr [n][3][t/scale][t/scale] fp32, all
 * contiguous; scale in {2, 3, 4}, t % scale == 0; Normalize(v) = (v/255 - mean[c]) / std[c]. */
typedef struct isr_sr_transform_desc {
    const uint8_t* crops;
    float* hr;
    float* lr;
    int32_t n, t, scale, hr_norm;
    float mean[3], std[3];
} isr_sr_transform_desc;
int isr_sr_transform(const isr_sr_transform_desc* d, isr_stream_t s);

/* Layout conversion between NCHW fp32 tensors and channel-blocked views
 * (network / loss boundaries: the VGG19 input, utils/loss.py:16-24, and the
 * gradient it receives).  to_blocked writes channels [0, round16(c)) of v (zeros
 * past c and outside the valid region), v = x*scale[c] + shift[c] (NULL → 1 / 0),
 * then the optional LeakyReLU' mask m (ReLU' with mslope 0); to_nchw reads
 * channels [0, c) of v into nchw, applying scale/shift. */
typedef struct isr_convert_desc {
    int32_t n, h, w, ha, wa, c;
    void* nchw;
    isr_view v;
    const float* scale;
    const float* shift;
    isr_view m;
    float mslope;
} isr_convert_desc;
int isr_nchw_to_blocked(const isr_convert_desc* d, isr_stream_t s);
int isr_blocked_to_nchw(const isr_convert_desc* d, isr_stream_t s);

/* 2x2 stride-2 max pool (torchvision vgg19.features MaxPool2d, used by
 * TruncatedVGG19 utils/models.py:454-510).  Input grid h x w (even), output
 * (h/2) x (w/2) with computed region hao x wao (multiples of 32).
 * fwd: y = maxpool(x).  bwd: g (input grid) = y (output gradient) routed to the
 * first maximum of each window, times (x > 0 ? 1 : mslope). */
typedef struct isr_pool_desc {
    int32_t n, h, w, c, hao, wao;
    isr_view x, y, g;
    float mslope;
} isr_pool_desc;
int isr_maxpool2_fwd(const isr_pool_desc* d, isr_stream_t s);
int isr_maxpool2_bwd(const isr_pool_desc* d, isr_stream_t s);

/* Train-mode BatchNorm2d (the `bn` of Conv, utils/models.py:75-111, trained by
 * train.py with ResNet; nn.BatchNorm2d semantics: biased batch variance for the
 * normalisation, unbiased for running_var, momentum update), on channel-blocked
 * views of c channels.  Statistics accumulate in acc[2][c] (double, caller-zeroed
 * before each reduce); finalize writes save[2][c] = (mean, 1/sqrt(var + eps)).
 *   isr_bn_stats      acc += (sum z, sum z^2)
 *   isr_bn_finalize   save, running_mean / running_var update
 *   isr_bn_apply      y = ((LeakyReLU_slope(a z + b)) * s1 + r1) * s2 + r2,  a = gamma * invstd,
 *                     b = beta - mean * a  (r1 / r2 optional; zero outside the valid region)
 *   isr_bn_bwd_reduce acc += (sum g, sum g * xhat),  g = y view (gradient wrt the BN output)
 *   isr_bn_bwd_apply  dz = gscale * a * (g - mean(g) - xhat * mean(g xhat))  into dz (or over y when
 *                     dz.data == NULL); dgamma = gscale * sum(g xhat), dbeta = gscale * sum(g) */
typedef struct isr_bn_desc {
    int32_t n, h, w, ha, wa, c;
    isr_view z, y, r1, r2, dz;
    float s1, s2, slope;
    const float* gamma;
    const float* beta;
    float* running_mean;      /* NULL: no running-stat update */
    float* running_var;
    float momentum, eps;
    double* acc;
    float* save;
    float* dgamma;
    float* dbeta;
    float gscale;
} isr_bn_desc;
int isr_bn_stats(const isr_bn_desc* d, isr_stream_t s);
int isr_bn_finalize(const isr_bn_desc* d, isr_stream_t s);
int isr_bn_apply(const isr_bn_desc* d, isr_stream_t s);
int isr_bn_bwd_reduce(const isr_bn_desc* d, isr_stream_t s);
int isr_bn_bwd_apply(const isr_bn_desc* d, isr_stream_t s);

/* Weight packing (device fp32 OIHW → device bf16 kernel layout).  Replaces the
 * one-off fuse step's weight preparation (utils/models.py:741-751); BN folding
 * itself is done by the caller before packing. */
size_t isr_conv3x3_packed_bytes(int32_t cout, int32_t cin);
int isr_pack_conv3x3(const float* w_oihw, void* packed, int32_t cout, int32_t cin, isr_stream_t s);
/* Input-gradient (dgrad) packing of a layer's [cout][cin][3][3] weights: the
 * result is an isr_conv3x3_fwd weight set for the conv cout → cin with the
 * kernel rotated by 180° and multiplied by `scale` (isr_conv3x3_packed_bytes(cin,
 * cout) bytes).  sub2 = 1 orders its input channels for isr_conv_desc.x_sub2
 * (the Scaler backward, utils/models.py:583). */
int isr_pack_conv3x3_dgrad(const float* w_oihw, void* packed, int32_t cout, int32_t cin, float scale, int32_t sub2,
                           isr_stream_t s);
/* Many isr_pack_conv3x3 / isr_pack_conv3x3_dgrad in one launch (items: device array). */
typedef struct isr_pack_item {
    const float* w; /* layer weights [cout][cin][3][3] fp32 (dgrad with src_cin > 0: [cout][src_cin][3][3]) */
    void* out;      /* packed bf16, isr_conv3x3_packed_bytes(cout, cin) bytes */
    int32_t cout, cin;
    int32_t dgrad;  /* 0: forward pack; 1: dgrad pack (as isr_pack_conv3x3_dgrad) */
    int32_t sub2;
    float scale;
    /* dgrad window (0, 0 = the whole layer): pack only the layer's input channels
     * [src_n0, src_n0 + cin) of a layer with src_cin input channels, i.e. the slice of the
     * transposed conv that produces those channels.  `out` may point inside a larger pack: a
     * conv whose input concatenates several layers' output gradients (the RDB input-gradient
     * "gather" convs of the training backward) is packed as one item per input block, at
     * packed offset (block's first input channel / 16) * 9 * cin * 16 elements. */
    int32_t src_n0, src_cin;
    int32_t pad_;
} isr_pack_item;
int isr_pack_conv3x3_batch(const isr_pack_item* items, int32_t n, isr_stream_t s);
size_t isr_head9x9_packed_bytes(int32_t cout, int32_t cin);
int isr_pack_head9x9(const float* w_oihw, void* packed, int32_t cout, int32_t cin, isr_stream_t s);
size_t isr_tail9x9_packed_bytes(int32_t cout, int32_t cin);
int isr_pack_tail9x9(const float* w_oihw, void* packed, int32_t cout, int32_t cin, isr_stream_t s);
/* The same three packs in fp16 (same layouts and sizes), for descriptors with f16 = 1. */
int isr_pack_conv3x3_f16(const float* w_oihw, void* packed, int32_t cout, int32_t cin, isr_stream_t s);
int isr_pack_head9x9_f16(const float* w_oihw, void* packed, int32_t cout, int32_t cin, isr_stream_t s);
int isr_pack_tail9x9_f16(const float* w_oihw, void* packed, int32_t cout, int32_t cin, isr_stream_t s);

int isr_conv3x3_fwd(const isr_conv_desc* d, isr_stream_t s);
/* Tuning entry point: same contract as isr_conv3x3_fwd with an explicit kernel
 * variant (0 = the production choice).  The production library carries variant 0
 * only; the tile / pipeline alternatives (1-3, 8, 9) and the timing-only ablations
 * (4-7) exist in a library built with -DISR_TUNING (lib/libisr_tuning.so).  Every
 * non-ablation variant writes the same outputs as variant 0 (up to fp32 summation
 * order).  Returns ISR_ERR_UNSUPPORTED for a variant this library does not carry. */
int isr_conv3x3_fwd_variant(const isr_conv_desc* d, int32_t variant, isr_stream_t s);
/* Tuning builds (-DISR_TUNING) only: per-block wall-clock stamps of later conv3x3
 * launches into `buf` (8 x uint64 per block: entry, first chunk landed, main loop
 * done, epilogue done [s_memrealtime, 100 MHz], -, -, HW_ID, XCC_ID); NULL stops.
 * A default build returns ISR_ERR_UNSUPPORTED. */
int isr_tuning_conv_stamps(void* buf);
/* Tuning builds only: per-wave stamps of later row-streaming tail launches (tail variant
 * 36 = 4 with stamps) into `buf` (4 x uint64 per (block, wave): entry, exit, summed
 * top-of-row-group wait + barrier, summed loop; s_memrealtime ticks); NULL stops. */
int isr_tuning_tail_stamps(void* buf);
/* Tuning builds only: persistent-chain probes for later isr_conv_chain launches —
 * workgroups with bit `delay_shift` of their index set start `delay_ticks` (100 MHz) late;
 * k2 = chain kernel variant for later launches (0 = production; A/B only); k3 reserved (0).
 * A default build returns ISR_ERR_UNSUPPORTED. */
int isr_tuning_chain_knobs(int32_t delay_ticks, int32_t delay_shift, int32_t k2, int32_t k3);
/* Validation only: ISR_OK when isr_conv3x3_fwd would accept `d` (nothing launched). */
int isr_conv3x3_check(const isr_conv_desc* d);

/* Persistent chain of RDB convs (the RRDB trunk, utils/models.py:245-317) in ONE launch:
 * layer i is layers[i] (device memory), each a descriptor isr_conv3x3_check accepts, of
 * kind kinds[i]: 0 = growth conv (cout 32), 1 = RDB final conv (cin 192, cout 64); all
 * layers share n, ha, wa (plain 3x3, no x_sub2 / taps / shuffle / mask).  Replaces nl
 * isr_conv3x3_fwd calls with the same outputs.  Tiles of layer i start as soon as their
 * 3x3 tile neighbourhood of layer i-1 is done (tile-level dependencies, no grid barrier).
 * `state` (device, isr_conv_chain_state_words(n, ha, wa) uint32 words, zeroed ONCE by the
 * caller before first use, then owned by the library across calls: a generation counter in
 * state[0] replaces per-call zeroing); after a call, state[1] == state[0] means a dependency
 * wait gave up (results invalid — not expected unless the device is shared); state[2] is a
 * sticky give-up counter that only grows (never reset): ANY change since the last value a host
 * saw means a launch in between gave up (one add per giving-up wave or refused launch, so it
 * is not a count of failed launches); state[3] belongs to the host (the library never writes it:
 * isr_mt_adam_guarded / isr_mt_lerp_guarded compare it with state[2]).  1 <= nl <= 1024.
 * acquire = 1 adds an agent-scope acquire before each tile's loads (otherwise the
 * hand-off relies on sc1 loads). */
typedef struct isr_chain_desc {
    const isr_conv_desc* layers;
    const int32_t* kinds;
    int32_t nl;
    int32_t n, ha, wa;
    uint32_t* state;
    int32_t acquire;
    int32_t f16;    /* every layer's isr_conv_desc.f16 (the table lives in device memory): 1 = fp16 */
} isr_chain_desc;
size_t isr_conv_chain_state_words(int32_t n, int32_t ha, int32_t wa);
int isr_conv_chain(const isr_chain_desc* c, isr_stream_t s);
/* The same with the kernel chosen: 0 = production (trunk.hip: one continuous K-chunk stream per
 * workgroup across its (layer, tile) items, waits only before the chunks the previous layer
 * wrote, the RDB residual folded into the MFMAs; needs every view to share (hp, wp, cs, pad),
 * a bias, cin >= 64, r1 (if any) == the layer's own input with slope 1 and 1/s1 exact in the storage type (bf16, or fp16 with f16) —
 * a table that breaks this makes the launch give up: state[1] == state[0]); 1 = the round-2
 * kernel (conv3x3.hip: one independent conv tile per (layer, tile)).  Both produce the outputs
 * of the per-layer isr_conv3x3_fwd calls bit for bit.  0 = trunk.hip in its two-workgroups-per-CU
 * form (4 waves of 4 output rows each, one K-chunk in flight); 2 = trunk.hip with one 8-wave
 * workgroup per CU (2 output rows per wave) and three chunks in flight; 3 = trunk.hip on 32x32
 * tiles, one 8-wave workgroup per CU (4 rows per wave; needs ha % 32 == 0); 5 = trunk.hip's
 * pair tile and ring with two 8-wave workgroups per CU (2 rows per wave, 4 waves per SIMD at
 * 128 VGPRs: one fragment set read a kernel row ahead, half the refill pieces per wave); 6 = the
 * production form with an XCD-aware tile deal (each XCD streams a contiguous range of tiles); 7 / 8 =
 * the production form with non-temporal halo loads / output stores.  Variants 4 (the deep-ring form,
 * round 4) and 9 (the loader / consumer form, round 5) measured slower and were removed in round 6
 * (ISR_ERR_UNSUPPORTED; their numbers stay in DESIGN.md §5).  The production library carries
 * variant 0 only (every other variant measured slower); variants 1-3 and 5-8 are
 * built into the tuning library (-DISR_TUNING) and return ISR_ERR_UNSUPPORTED here. */
int isr_conv_chain_variant(const isr_chain_desc* c, int32_t variant, isr_stream_t s);
/* Tuning builds only: per (layer 75..89, tile) stamps of later production chain launches into
 * `buf` (8 x uint64: entry, chunk 0 landed, main loop done, stores issued, deferred wait start,
 * wait met; s_memrealtime ticks, 100 MHz); NULL stops. */
int isr_tuning_trunk_stamps(void* buf);
/* Tuning builds only: ablations of later production chain launches (timing only, outputs wrong):
 * bit 1 = no halo LDS-DMA, 4 = no epilogue stores, 8 = no weight LDS-DMA, 16 = no dependency
 * waits;
 * per_cu > 0 caps the resident workgroups per CU (the grid). */
int isr_tuning_trunk_knobs(int32_t ablate, int32_t per_cu, int32_t k2, int32_t k3);
/* Tuning builds only: per-item cycle stamps (s_memtime) of later production chain launches into
 * `buf` (uint64 [grid][2 layers: 77, 79][16 items][2 waves][8]: item top, own DMA landed, barrier
 * passed, refill issued, MFMAs issued) for each workgroup's first tile; NULL stops. */
int isr_tuning_trunk_item_stamps(void* buf);

int isr_head9x9_fwd(const isr_head_desc* d, isr_stream_t s);
int isr_tail9x9_fwd(const isr_tail_desc* d, isr_stream_t s);
/* Tuning / A-B entry point: 0 = production (= 5), 1 = one 16-row tile per block, 3 = one
 * 8-row tile per block (76 KB LDS, 2 blocks / CU), 2 = persistent (one block per CU, streamed
 * halo ring), 4 = row-streaming walk down a 32-column strip (4 waves, each T row computed
 * once), 5 = the same walk with 8 waves (two per SIMD), 6 = lane-streaming walk (one wave per
 * strip, running ky sums shifted one lane per row).  All bit-identical.  The production
 * library carries 0, 3 (the fallback for outputs past 2 GiB) and 5; 1, 2, 4 and 6 are in the
 * tuning library (-DISR_TUNING) only (ISR_ERR_UNSUPPORTED here).
 * Same descriptor rules as isr_tail9x9_fwd. */
int isr_tail9x9_fwd_variant(const isr_tail_desc* d, int32_t variant, isr_stream_t s);

/* ---- multi-tensor optimiser ops (one launch over every parameter) ---------
 * A tensor is n fp32 elements at each non-null pointer (same element order);
 * a chunk is elements [start, start + len) of tensor t.  The host builds the
 * tensor and chunk tables in device memory (len <= 65536 recommended).
 * Replaces: torch.optim.Adam.step (train.py:264-267, stepped at :58/:102/:118),
 * clip_grad_norm_(params, 10) (train.py:57, :101, :116), ModelEMA.update
 * (utils/models.py:31-40). */
typedef struct isr_mt_tensor {
    float* p; /* param (Adam), EMA tensor (lerp) */
    float* g; /* grad (Adam, sumsq, scale), model tensor (lerp) */
    float* m; /* exp_avg */
    float* v; /* exp_avg_sq */
    int64_t n;
} isr_mt_tensor;

typedef struct isr_mt_chunk {
    int32_t t, len;
    int64_t start;
} isr_mt_chunk;

/* torch.optim.Adam (amsgrad=False, maximize=False): g' = g*scale (+ wd*p);
 * m = lerp(m, g', 1-beta1); v = beta2*v + (1-beta2)*g'^2;
 * p += step * m / (sqrt(v)/bc2_sqrt + eps), step = -lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t). */
typedef struct isr_adam_args {
    float step, beta1, beta2, eps, weight_decay, bc2_sqrt;
} isr_adam_args;

/* `scale` (device, nullable): gradient multiplier applied on the fly (e.g. a clip coefficient). */
int isr_mt_adam(const isr_mt_tensor* tensors, const isr_mt_chunk* chunks, int32_t nchunks, const isr_adam_args* a,
                const float* scale, isr_stream_t s);
/* partial[k] = sum of g^2 over chunk k. */
int isr_mt_sumsq(const isr_mt_tensor* tensors, const isr_mt_chunk* chunks, int32_t nchunks, float* partial,
                 isr_stream_t s);
/* out[0] = sqrt(sum partial), out[1] = min(1, max_norm / (out[0] + 1e-6)) — clip_grad_norm_'s coefficient. */
int isr_clip_coef(const float* partial, int32_t n, float max_norm, float* out, isr_stream_t s);
/* g *= *coef over every chunk (clip_grad_norm_'s in-place scaling). */
int isr_mt_scale(const isr_mt_tensor* tensors, const isr_mt_chunk* chunks, int32_t nchunks, const float* coef,
                 isr_stream_t s);
/* p = p*d + (1-d)*g over every chunk (ModelEMA.update: p = EMA tensor, g = model tensor). */
int isr_mt_lerp(const isr_mt_tensor* tensors, const isr_mt_chunk* chunks, int32_t nchunks, float d, isr_stream_t s);
/* The same two updates, skipped on the device (no host synchronisation) when guard[0] != guard[1]:
 * pass `isr_chain_desc.state + 2` of the trunk launch that produced this step's forward (state[2]
 * the sticky give-up counter, state[3] the count the host has accepted, zero-initialised with the
 * state), so a forward whose dependency wait gave up never reaches the parameters or the EMA.
 * guard = NULL is the unguarded call. */
int isr_mt_adam_guarded(const isr_mt_tensor* tensors, const isr_mt_chunk* chunks, int32_t nchunks,
                        const isr_adam_args* a, const float* scale, const uint32_t* guard, isr_stream_t s);
int isr_mt_lerp_guarded(const isr_mt_tensor* tensors, const isr_mt_chunk* chunks, int32_t nchunks, float d,
                        const uint32_t* guard, isr_stream_t s);

const char* isr_last_error(void);
int isr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ISR_H */
