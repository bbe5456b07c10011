// extern "C" entry points of libisr.so (declared in include/isr.h).
// Validation happens here so that a bad descriptor never reaches a kernel:
// every kernel indexes its tiles without bounds checks.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "isr_common.h"

namespace isr {
int conv3x3_fwd_dispatch(const isr_conv_desc* d, hipStream_t s);
int conv3x3_fwd_variant(const isr_conv_desc* d, int variant, hipStream_t s);
int conv_stamps_set(void* p);
int chain_knobs_set(const int* k);
int tail_stamps_set(void* p);
size_t conv_chain_state_words(int n, int ha, int wa);
int conv_chain(const isr_chain_desc* c, hipStream_t s);
size_t trunk_state_words(int n, int ha, int wa);
int trunk_launch(const isr_chain_desc* c, hipStream_t s, int form);
int trunk_stamps_set(void* p);
int trunk_knobs_set(const int* k);
int trunk_item_stamps_set(void* p);
size_t conv3x3_packed_bytes(int cout, int cin);
int conv3x3_pack(const float* w, void* out, int cout, int cin, hipStream_t s);
int conv3x3_pack_f16(const float* w, void* out, int cout, int cin, hipStream_t s);
int head9x9_fwd_dispatch(const isr_head_desc* d, hipStream_t s);
int tail9x9_fwd_dispatch(const isr_tail_desc* d, hipStream_t s);
int tail9x9_fwd_variant(const isr_tail_desc* d, int variant, hipStream_t s);
size_t head9x9_packed_bytes(int cout);
size_t tail9x9_packed_bytes();
int head9x9_pack(const float* w, void* out, int cout, int cin, hipStream_t s, bool h);
int tail9x9_pack(const float* w, void* out, int cout, int cin, hipStream_t s, bool h);
int conv3x3_pack_dgrad(const float* w, void* out, int cout, int cin, float scale, int sub2, hipStream_t s);
int conv3x3_pack_batch(const isr_pack_item* items, int n, hipStream_t s);
int ew_combine_dispatch(const isr_ew_desc* d, hipStream_t s);
int pixel_shuffle2_dispatch(const isr_ew_desc* d, hipStream_t s);
int sr_transform_dispatch(const isr_sr_transform_desc* d, hipStream_t s);
int pixel_unshuffle2_dispatch(const isr_ew_desc* d, hipStream_t s);
int bn_dispatch(const isr_bn_desc* d, int op, hipStream_t s);
int nchw_to_blocked_dispatch(const isr_convert_desc* d, hipStream_t s);
int blocked_to_nchw_dispatch(const isr_convert_desc* d, hipStream_t s);
int maxpool2_dispatch(const isr_pool_desc* d, int backward, hipStream_t s);
size_t wgrad3x3_workspace_bytes(const isr_wgrad_desc* d, int variant);
size_t wgrad9x9_workspace_bytes(const isr_wgrad9_desc* d);
int wgrad9x9_dispatch(const isr_wgrad9_desc* d, void* ws, size_t ws_bytes, hipStream_t s);
int wgrad3x3_dispatch(const isr_wgrad_desc* d, int variant, void* ws, size_t ws_bytes, hipStream_t s, int parts);
size_t wgrad3x3_group_workspace_bytes(const isr_wgrad_desc* ds, int n, int variant);
int wgrad3x3_group_dispatch(const isr_wgrad_desc* ds, int n, void* ws, size_t ws_bytes, hipStream_t s, int variant);
int mt_adam_dispatch(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int n, const isr_adam_args* a,
                     const float* scale, const uint32_t* guard, hipStream_t s);
int mt_sumsq_dispatch(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int n, float* partial, hipStream_t s);
int clip_coef_dispatch(const float* partial, int n, float max_norm, float* out, hipStream_t s);
int mt_axpby_dispatch(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int n, int mode, const float* coef, float d,
                      const uint32_t* guard, hipStream_t s);
}  // namespace isr

static thread_local char g_err[512] = "";

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

static int launched(int rc, const char* what) {
    if (rc != 0) {
        hipError_t e = hipGetLastError();
        return fail(ISR_ERR_LAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
    }
    g_err[0] = 0;
    return ISR_OK;
}

// A view must hold rows [-halo, ha + halo) and cols [-halo, wa + halo) of the
// computed region plus `ch` channels from coff.
static bool view_ok(const isr_view& v, int ha, int wa, int halo, int ch, const char* name, int align16) {
    if (!v.data) { fail(ISR_ERR_BAD_DESC, "%s: null data", name); return false; }
    if (v.pad < halo) { fail(ISR_ERR_BAD_DESC, "%s: pad %d < required halo %d", name, v.pad, halo); return false; }
    if (v.hp < ha + 2 * v.pad || v.wp < wa + 2 * v.pad) {
        fail(ISR_ERR_BAD_DESC, "%s: buffer %dx%d (pad %d) smaller than computed region %dx%d", name, v.hp, v.wp, v.pad, ha, wa);
        return false;
    }
    if (v.coff < 0 || v.coff + ch > v.cs) {
        fail(ISR_ERR_BAD_DESC, "%s: channels [%d,%d) exceed stride %d", name, v.coff, v.coff + ch, v.cs);
        return false;
    }
    if (align16 && ((v.cs % 16) || (v.coff % 16) || ((uintptr_t)v.data % 16))) {
        fail(ISR_ERR_BAD_DESC, "%s: channel count/offset must be multiples of 16 (channel-blocked layout) "
             "and data 16-byte aligned", name);
        return false;
    }
    return true;
}

extern "C" {

const char* isr_last_error(void) { return g_err; }

int isr_pack_conv3x3_batch(const isr_pack_item* items, int32_t n, isr_stream_t s) {
    if (!items || n <= 0 || n > 65535) return fail(ISR_ERR_BAD_DESC, "pack_conv3x3_batch: bad item table (n=%d)", n);
    return launched(isr::conv3x3_pack_batch(items, n, (hipStream_t)s), "pack_conv3x3_batch");
}

static int mt_ok(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, const char* what) {
    if (!ts || !cs) return fail(ISR_ERR_BAD_DESC, "%s: null tensor / chunk table", what);
    if (n <= 0 || n > (1 << 30)) return fail(ISR_ERR_BAD_DESC, "%s: bad chunk count %d", what, n);
    return ISR_OK;
}

int isr_mt_adam_guarded(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, const isr_adam_args* a,
                        const float* scale, const uint32_t* guard, isr_stream_t s) {
    if (int rc = mt_ok(ts, cs, n, "mt_adam")) return rc;
    if (!a) return fail(ISR_ERR_BAD_DESC, "mt_adam: null args");
    if (!(a->bc2_sqrt > 0.f) || !(a->beta1 >= 0.f && a->beta1 < 1.f) || !(a->beta2 >= 0.f && a->beta2 < 1.f))
        return fail(ISR_ERR_BAD_DESC, "mt_adam: bad betas / bias correction");
    return launched(isr::mt_adam_dispatch(ts, cs, n, a, scale, guard, (hipStream_t)s), "mt_adam");
}

int isr_mt_adam(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, const isr_adam_args* a,
                const float* scale, isr_stream_t s) {
    return isr_mt_adam_guarded(ts, cs, n, a, scale, nullptr, s);
}

int isr_mt_sumsq(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, float* partial, isr_stream_t s) {
    if (int rc = mt_ok(ts, cs, n, "mt_sumsq")) return rc;
    if (!partial) return fail(ISR_ERR_BAD_DESC, "mt_sumsq: null partial buffer");
    return launched(isr::mt_sumsq_dispatch(ts, cs, n, partial, (hipStream_t)s), "mt_sumsq");
}

int isr_clip_coef(const float* partial, int32_t n, float max_norm, float* out, isr_stream_t s) {
    if (!partial || !out || n <= 0) return fail(ISR_ERR_BAD_DESC, "clip_coef: bad arguments");
    return launched(isr::clip_coef_dispatch(partial, n, max_norm, out, (hipStream_t)s), "clip_coef");
}

int isr_mt_scale(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, const float* coef, isr_stream_t s) {
    if (int rc = mt_ok(ts, cs, n, "mt_scale")) return rc;
    if (!coef) return fail(ISR_ERR_BAD_DESC, "mt_scale: null coefficient");
    return launched(isr::mt_axpby_dispatch(ts, cs, n, 0, coef, 0.f, nullptr, (hipStream_t)s), "mt_scale");
}

int isr_mt_lerp_guarded(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, float d, const uint32_t* guard,
                        isr_stream_t s) {
    if (int rc = mt_ok(ts, cs, n, "mt_lerp")) return rc;
    return launched(isr::mt_axpby_dispatch(ts, cs, n, 1, nullptr, d, guard, (hipStream_t)s), "mt_lerp");
}

int isr_mt_lerp(const isr_mt_tensor* ts, const isr_mt_chunk* cs, int32_t n, float d, isr_stream_t s) {
    return isr_mt_lerp_guarded(ts, cs, n, d, nullptr, s);
}
int isr_version(void) { return 1; }

size_t isr_conv3x3_packed_bytes(int32_t cout, int32_t cin) { return isr::conv3x3_packed_bytes(cout, cin); }
size_t isr_head9x9_packed_bytes(int32_t cout, int32_t cin) { (void)cin; return isr::head9x9_packed_bytes(cout); }
size_t isr_tail9x9_packed_bytes(int32_t cout, int32_t cin) { (void)cout; (void)cin; return isr::tail9x9_packed_bytes(); }

int isr_pack_conv3x3(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s) {
    if (!w || !packed) return fail(ISR_ERR_BAD_DESC, "pack_conv3x3: null pointer");
    if (cin <= 0 || cin % 16) return fail(ISR_ERR_UNSUPPORTED, "pack_conv3x3: cin %d must be a positive multiple of 16", cin);
    if (cout <= 0 || cout % 32)
        return fail(ISR_ERR_UNSUPPORTED, "pack_conv3x3: cout %d must be a positive multiple of 32", cout);
    return launched(isr::conv3x3_pack(w, packed, cout, cin, (hipStream_t)s), "pack_conv3x3");
}

int isr_pack_conv3x3_dgrad(const float* w, void* packed, int32_t cout, int32_t cin, float scale, int32_t sub2,
                           isr_stream_t s) {
    if (!w || !packed) return fail(ISR_ERR_BAD_DESC, "pack_conv3x3_dgrad: null pointer");
    if (cin <= 0 || cin % 32 || cout <= 0 || cout % 32)
        return fail(ISR_ERR_UNSUPPORTED, "pack_conv3x3_dgrad: cin %d / cout %d must be multiples of 32", cin, cout);
    if (sub2 && cout % 128) return fail(ISR_ERR_UNSUPPORTED, "pack_conv3x3_dgrad: sub2 needs cout %% 128 == 0");
    return launched(isr::conv3x3_pack_dgrad(w, packed, cout, cin, scale, sub2, (hipStream_t)s), "pack_conv3x3_dgrad");
}

static int pack_head_any(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s, bool h) {
    if (!w || !packed) return fail(ISR_ERR_BAD_DESC, "pack_head9x9: null pointer");
    if (cout != 64 || cin < 1 || cin > 3) return fail(ISR_ERR_UNSUPPORTED, "pack_head9x9: need cout 64, cin <= 3 (got %d, %d)", cout, cin);
    return launched(isr::head9x9_pack(w, packed, cout, cin, (hipStream_t)s, h), "pack_head9x9");
}
int isr_pack_head9x9(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s) {
    return pack_head_any(w, packed, cout, cin, s, false);
}
int isr_pack_head9x9_f16(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s) {
    return pack_head_any(w, packed, cout, cin, s, true);
}

static int pack_tail_any(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s, bool h) {
    if (!w || !packed) return fail(ISR_ERR_BAD_DESC, "pack_tail9x9: null pointer");
    if (cout != 3 || cin != 64) return fail(ISR_ERR_UNSUPPORTED, "pack_tail9x9: need cout 3, cin 64 (got %d, %d)", cout, cin);
    return launched(isr::tail9x9_pack(w, packed, cout, cin, (hipStream_t)s, h), "pack_tail9x9");
}
int isr_pack_tail9x9(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s) {
    return pack_tail_any(w, packed, cout, cin, s, false);
}
int isr_pack_tail9x9_f16(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s) {
    return pack_tail_any(w, packed, cout, cin, s, true);
}

int isr_pack_conv3x3_f16(const float* w, void* packed, int32_t cout, int32_t cin, isr_stream_t s) {
    if (!w || !packed) return fail(ISR_ERR_BAD_DESC, "pack_conv3x3_f16: null pointer");
    if (cin <= 0 || cin % 16) return fail(ISR_ERR_UNSUPPORTED, "pack_conv3x3_f16: cin %d must be a positive multiple of 16", cin);
    if (cout <= 0 || cout % 32)
        return fail(ISR_ERR_UNSUPPORTED, "pack_conv3x3_f16: cout %d must be a positive multiple of 32", cout);
    return launched(isr::conv3x3_pack_f16(w, packed, cout, cin, (hipStream_t)s), "pack_conv3x3_f16");
}

static int conv3x3_validate(const isr_conv_desc* d) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "conv3x3: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0) return fail(ISR_ERR_BAD_DESC, "conv3x3: empty problem n=%d h=%d w=%d", d->n, d->h, d->w);
    if (d->ha % ISR_TILE_H || d->wa % ISR_TILE_W || d->ha < d->h || d->wa < d->w)
        return fail(ISR_ERR_BAD_DESC, "conv3x3: computed region %dx%d must cover %dx%d and be a multiple of %dx%d", d->ha, d->wa,
                    d->h, d->w, ISR_TILE_H, ISR_TILE_W);
    if (d->cin <= 0 || d->cin % 16) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: cin %d must be a multiple of 16", d->cin);
    if (d->cout <= 0 || d->cout % 32)
        return fail(ISR_ERR_UNSUPPORTED, "conv3x3: cout %d must be a positive multiple of 32", d->cout);
    if (!d->wpack) return fail(ISR_ERR_BAD_DESC, "conv3x3: null weights");
    if (d->shuffle != 1 && d->shuffle != 2) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: shuffle must be 1 or 2");
    if (d->taps < 0 || d->taps > 2) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: taps must be 0, 1 or 2");
    if (d->taps && d->cout % 64) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: a 2x2 tap window needs cout %% 64 == 0");
    if (d->x_sub2) {
        if (d->cin % 128) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: x_sub2 needs cin %% 128 == 0 (got %d)", d->cin);
        if (d->shuffle != 1) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: x_sub2 with a shuffled store");
        if (!view_ok(d->x, 2 * d->ha, 2 * d->wa, 2, d->cin / 4, "conv3x3.x", 1)) return ISR_ERR_BAD_DESC;
    } else if (!view_ok(d->x, d->ha, d->wa, 1, d->cin, "conv3x3.x", 1)) {
        return ISR_ERR_BAD_DESC;
    }
    if (d->m.data) {
        if (d->y2.data) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: mask epilogue takes no second output");
        if (d->m_c0 < 0 || d->m_c0 % 32) return fail(ISR_ERR_BAD_DESC, "conv3x3: m_c0 %d must be a multiple of 32", d->m_c0);
        if (d->shuffle == 2) {  // mask read on the shuffled (2h x 2w) grid, every channel
            if (d->m_c0) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: a shuffled store masks all channels (m_c0 = 0)");
            if (!view_ok(d->m, 2 * d->ha, 2 * d->wa, 0, d->cout / 4, "conv3x3.m", 1)) return ISR_ERR_BAD_DESC;
        } else if (!view_ok(d->m, d->ha, d->wa, 0, d->cout, "conv3x3.m", 1)) {
            return ISR_ERR_BAD_DESC;
        }
    }
    if (d->r1_cn < 0 || d->r1_cn % 32) return fail(ISR_ERR_BAD_DESC, "conv3x3: r1_cn %d must be a multiple of 32", d->r1_cn);
    if (d->shuffle == 2) {
        if (d->cout % 64) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: pixel shuffle needs cout %% 64 == 0");
        if (d->r1.data || d->r2.data || d->y2.data)
            return fail(ISR_ERR_UNSUPPORTED, "conv3x3: pixel shuffle store takes no residual / second output");
        if (!view_ok(d->y, 2 * d->ha, 2 * d->wa, 0, d->cout / 4, "conv3x3.y", 1)) return ISR_ERR_BAD_DESC;
    } else {
        if (!view_ok(d->y, d->ha, d->wa, 0, d->cout, "conv3x3.y", 1)) return ISR_ERR_BAD_DESC;
        if (d->y2.data && !view_ok(d->y2, d->ha, d->wa, 0, d->cout, "conv3x3.y2", 1)) return ISR_ERR_BAD_DESC;
        if (d->r1.data && !view_ok(d->r1, d->ha, d->wa, 0, d->cout, "conv3x3.r1", 1)) return ISR_ERR_BAD_DESC;
        if (d->r2.data && !view_ok(d->r2, d->ha, d->wa, 0, d->cout, "conv3x3.r2", 1)) return ISR_ERR_BAD_DESC;
    }
    if (d->bias && ((uintptr_t)d->bias % 16)) return fail(ISR_ERR_BAD_DESC, "conv3x3: bias must be 16-byte aligned");
    if (d->f16 != 0 && d->f16 != 1) return fail(ISR_ERR_BAD_DESC, "conv3x3: f16 must be 0 or 1");
    if (d->f16 && (d->m.data || d->x_sub2 || d->taps))
        return fail(ISR_ERR_UNSUPPORTED, "conv3x3: fp16 activations are forward-only (no mask, x_sub2 or tap window)");
    return ISR_OK;
}

int isr_conv3x3_fwd(const isr_conv_desc* d, isr_stream_t s) {
    int rc = conv3x3_validate(d);
    if (rc != ISR_OK) return rc;
    return launched(isr::conv3x3_fwd_dispatch(d, (hipStream_t)s), "conv3x3");
}

int isr_conv3x3_check(const isr_conv_desc* d) { return conv3x3_validate(d); }

size_t isr_conv_chain_state_words(int32_t n, int32_t ha, int32_t wa) {
    if (n <= 0 || ha <= 0 || wa <= 0 || ha % 16 || wa % 32) return 0;
    const size_t a = isr::conv_chain_state_words(n, ha, wa), b = isr::trunk_state_words(n, ha, wa);
    return a > b ? a : b;
}

int isr_conv_chain_variant(const isr_chain_desc* c, int32_t variant, isr_stream_t s) {
    if (!c || !c->layers || !c->kinds || !c->state || c->nl <= 0 || c->nl > 1024)
        return fail(ISR_ERR_BAD_DESC, "conv chain: null layers / kinds / state or nl not in [1, 1024]");
    if (c->n <= 0 || c->ha <= 0 || c->wa <= 0 || c->ha % 16 || c->wa % 32)
        return fail(ISR_ERR_BAD_DESC, "conv chain: bad grid n=%d ha=%d wa=%d", c->n, c->ha, c->wa);
    if (c->f16 != 0 && c->f16 != 1) return fail(ISR_ERR_BAD_DESC, "conv chain: f16 must be 0 or 1");
    if (c->f16 && variant != 0)
        return fail(ISR_ERR_UNSUPPORTED, "conv chain: fp16 storage runs the production trunk form (variant 0) only");
    if (variant == 4 || variant == 9)
        return fail(ISR_ERR_UNSUPPORTED, "conv chain: variant %d (a losing A/B form) was removed in round 6", variant);
    if (variant == 0 || (variant >= 2 && variant <= 8)) {
        static const int form_of[10] = {0, 0, 1, 2, 3, 4, 5, 6, 7, 8};
        const int rc = isr::trunk_launch(c, (hipStream_t)s, form_of[variant]);
        if (rc == -3) return fail(ISR_ERR_UNSUPPORTED, "conv chain: variant %d is an A/B form of the tuning library "
                                  "(lib/libisr_tuning.so)", variant);
        if (rc == -4) return fail(ISR_ERR_LAUNCH, "conv chain: the occupancy query admits no workgroup per CU");
        if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "conv chain: unsupported grid or layer count");
        return launched(rc, "conv chain");
    }
    if (variant == 1) {
        const int rc = isr::conv_chain(c, (hipStream_t)s);
        if (rc == -3) return fail(ISR_ERR_UNSUPPORTED, "conv chain: variant 1 (the round-2 kernel) is in the tuning library only");
        return launched(rc, "conv chain (round-2 kernel)");
    }
    return fail(ISR_ERR_UNSUPPORTED, "conv chain: unknown variant %d", variant);
}

int isr_conv_chain(const isr_chain_desc* c, isr_stream_t s) { return isr_conv_chain_variant(c, 0, s); }

int isr_tuning_trunk_knobs(int32_t ablate, int32_t per_cu, int32_t k2, int32_t k3) {
    const int k[4] = {ablate, per_cu, k2, k3};
    const int rc = isr::trunk_knobs_set(k);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "trunk knobs: library built without -DISR_TUNING");
    return rc == 0 ? ISR_OK : fail(ISR_ERR_LAUNCH, "trunk knobs: hipMemcpyToSymbol failed");
}

int isr_tuning_trunk_item_stamps(void* buf) {
    const int rc = isr::trunk_item_stamps_set(buf);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "trunk item stamps: library built without -DISR_TUNING");
    return rc == 0 ? ISR_OK : fail(ISR_ERR_LAUNCH, "trunk item stamps: hipMemcpyToSymbol failed");
}

int isr_tuning_trunk_stamps(void* buf) {
    const int rc = isr::trunk_stamps_set(buf);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "trunk stamps: library built without -DISR_TUNING");
    return rc == 0 ? ISR_OK : fail(ISR_ERR_LAUNCH, "trunk stamps: hipMemcpyToSymbol failed");
}

int isr_tuning_conv_stamps(void* buf) {
    const int rc = isr::conv_stamps_set(buf);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "conv stamps: library built without -DISR_TUNING");
    return rc == 0 ? ISR_OK : fail(ISR_ERR_LAUNCH, "conv stamps: hipMemcpyToSymbol failed");
}

int isr_tuning_chain_knobs(int32_t delay_ticks, int32_t delay_shift, int32_t k2, int32_t k3) {
    const int k[4] = {delay_ticks, delay_shift, k2, k3};
    const int rc = isr::chain_knobs_set(k);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "chain knobs: library built without -DISR_TUNING");
    return rc == 0 ? ISR_OK : fail(ISR_ERR_LAUNCH, "chain knobs: hipMemcpyToSymbol failed");
}

int isr_tuning_tail_stamps(void* buf) {
    const int rc = isr::tail_stamps_set(buf);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "tail stamps: library built without -DISR_TUNING");
    return rc == 0 ? ISR_OK : fail(ISR_ERR_LAUNCH, "tail stamps: hipMemcpyToSymbol failed");
}

int isr_conv3x3_fwd_variant(const isr_conv_desc* d, int32_t variant, isr_stream_t s) {
    int rc = conv3x3_validate(d);
    if (rc != ISR_OK) return rc;
    rc = isr::conv3x3_fwd_variant(d, variant, (hipStream_t)s);
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "conv3x3: variant %d not available for cout %d / cin %d", variant, d->cout, d->cin);
    return launched(rc, "conv3x3");
}

int isr_head9x9_fwd(const isr_head_desc* d, isr_stream_t s) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "head9x9: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0) return fail(ISR_ERR_BAD_DESC, "head9x9: empty problem");
    if (d->ha % ISR_TILE_H || d->wa % ISR_TILE_W || d->ha < d->h || d->wa < d->w)
        return fail(ISR_ERR_BAD_DESC, "head9x9: bad computed region %dx%d for %dx%d", d->ha, d->wa, d->h, d->w);
    if (d->cout != 64) return fail(ISR_ERR_UNSUPPORTED, "head9x9: cout must be 64");
    if (!d->x || !d->wpack) return fail(ISR_ERR_BAD_DESC, "head9x9: null input or weights");
    if (!view_ok(d->y, d->ha, d->wa, 0, 64, "head9x9.y", 1)) return ISR_ERR_BAD_DESC;
    if (d->y2.data && !view_ok(d->y2, d->ha, d->wa, 0, 64, "head9x9.y2", 1)) return ISR_ERR_BAD_DESC;
    if (d->m.data && !view_ok(d->m, d->ha, d->wa, 0, 64, "head9x9.m", 1)) return ISR_ERR_BAD_DESC;
    if (d->bias && ((uintptr_t)d->bias % 16)) return fail(ISR_ERR_BAD_DESC, "head9x9: bias must be 16-byte aligned");
    if (d->f16 != 0 && d->f16 != 1) return fail(ISR_ERR_BAD_DESC, "head9x9: f16 must be 0 or 1");
    if (d->f16 && d->m.data) return fail(ISR_ERR_UNSUPPORTED, "head9x9: fp16 activations are forward-only (no mask)");
    return launched(isr::head9x9_fwd_dispatch(d, (hipStream_t)s), "head9x9");
}

static int tail_validate(const isr_tail_desc* d) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "tail9x9: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0) return fail(ISR_ERR_BAD_DESC, "tail9x9: empty problem");
    if (d->ha % ISR_TILE_H || d->wa % ISR_TILE_W || d->ha < d->h || d->wa < d->w)
        return fail(ISR_ERR_BAD_DESC, "tail9x9: bad computed region %dx%d for %dx%d", d->ha, d->wa, d->h, d->w);
    if (d->cin != 64) return fail(ISR_ERR_UNSUPPORTED, "tail9x9: cin must be 64");
    if (!d->y || !d->wpack) return fail(ISR_ERR_BAD_DESC, "tail9x9: null output or weights");
    if (!view_ok(d->x, d->ha, d->wa, 4, 64, "tail9x9.x", 1)) return ISR_ERR_BAD_DESC;
    if (d->f16 != 0 && d->f16 != 1) return fail(ISR_ERR_BAD_DESC, "tail9x9: f16 must be 0 or 1");
    return ISR_OK;
}

int isr_tail9x9_fwd(const isr_tail_desc* d, isr_stream_t s) {
    const int rc = tail_validate(d);
    if (rc != ISR_OK) return rc;
    return launched(isr::tail9x9_fwd_dispatch(d, (hipStream_t)s), "tail9x9");
}

int isr_tail9x9_fwd_variant(const isr_tail_desc* d, int32_t variant, isr_stream_t s) {
    const int rc = tail_validate(d);
    if (rc != ISR_OK) return rc;
    const int r = isr::tail9x9_fwd_variant(d, variant, (hipStream_t)s);
    if (r == -2) return fail(ISR_ERR_UNSUPPORTED, "tail9x9: no variant %d", variant);
    return launched(r, "tail9x9");
}

static int wgrad_validate(const isr_wgrad_desc* d) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "wgrad3x3: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0) return fail(ISR_ERR_BAD_DESC, "wgrad3x3: empty problem");
    if (d->ha % ISR_TILE_H || d->wa % ISR_TILE_W || d->ha < d->h || d->wa < d->w)
        return fail(ISR_ERR_BAD_DESC, "wgrad3x3: bad computed region %dx%d for %dx%d", d->ha, d->wa, d->h, d->w);
    if (d->cin <= 0 || d->cin % 32 || d->cout <= 0 || d->cout % 32)
        return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: cin %d / cout %d must be multiples of 32", d->cin, d->cout);
    if (!d->dw) return fail(ISR_ERR_BAD_DESC, "wgrad3x3: null dw");
    if (d->splits < 0) return fail(ISR_ERR_BAD_DESC, "wgrad3x3: negative split count");
    if (d->taps < 0 || d->taps > 1) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: taps must be 0 or 1");
    if (d->x_sub2) {
        if (d->cin % 128) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: x_sub2 needs cin %% 128 == 0 (got %d)", d->cin);
        if (d->g_sub2) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: x_sub2 with g_sub2");
        if (!view_ok(d->x, 2 * d->ha, 2 * d->wa, 2, d->cin / 4, "wgrad3x3.x", 1)) return ISR_ERR_BAD_DESC;
    } else if (!view_ok(d->x, d->ha, d->wa, 1, d->cin, "wgrad3x3.x", 1)) {
        return ISR_ERR_BAD_DESC;
    }
    if (d->g_sub2) {
        if (d->cout % 128) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: g_sub2 needs cout %% 128 == 0");
        if (!view_ok(d->g, 2 * d->ha, 2 * d->wa, 0, d->cout / 4, "wgrad3x3.g", 1)) return ISR_ERR_BAD_DESC;
    } else if (!view_ok(d->g, d->ha, d->wa, 0, d->cout, "wgrad3x3.g", 1)) {
        return ISR_ERR_BAD_DESC;
    }
    return ISR_OK;
}

size_t isr_wgrad3x3_workspace_bytes(const isr_wgrad_desc* d) {
    if (wgrad_validate(d) != ISR_OK) return 0;
    return isr::wgrad3x3_workspace_bytes(d, 0);
}

// production: 0 and 16 (the compiler-read reference of the same tiles); tuning builds also 1-15
static bool wgrad_variant_built(int32_t variant) {
#ifdef ISR_TUNING
    return variant >= 0 && variant <= 16;
#else
    return variant == 0 || variant == 16;
#endif
}

static int wgrad3x3_parts(const isr_wgrad_desc* d, int32_t variant, void* workspace, size_t ws_bytes,
                          isr_stream_t s, int parts) {
    int rc = wgrad_validate(d);
    if (rc != ISR_OK) return rc;
    if (!workspace) return fail(ISR_ERR_BAD_DESC, "wgrad3x3: null workspace");
    if (!wgrad_variant_built(variant)) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: no variant %d in this library%s",
                                                   variant, variant >= 1 && variant <= 15 ? " (tuning form: build with "
                                                   "-DISR_TUNING)" : "");
    rc = isr::wgrad3x3_dispatch(d, variant, workspace, ws_bytes, (hipStream_t)s, parts);
    if (rc == -3) return fail(ISR_ERR_BAD_DESC, "wgrad3x3: workspace of %zu bytes is smaller than %zu", ws_bytes,
                              isr::wgrad3x3_workspace_bytes(d, variant));
    if (rc == -2)
        return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3: variant %d needs ha %% stage rows == 0 and cout / cin multiples "
                    "of its tile", variant);
    return launched(rc, "wgrad3x3");
}

int isr_wgrad3x3_variant(const isr_wgrad_desc* d, int32_t variant, void* workspace, size_t ws_bytes,
                         isr_stream_t s) {
    return wgrad3x3_parts(d, variant, workspace, ws_bytes, s, 3);
}

int isr_wgrad3x3(const isr_wgrad_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s) {
    return wgrad3x3_parts(d, 0, workspace, ws_bytes, s, 3);
}

static int wgrad_group_validate(const isr_wgrad_desc* ds, int32_t n) {
    if (!ds || n < 1 || n > 5) return fail(ISR_ERR_BAD_DESC, "wgrad3x3 group: null descriptors or n not in [1, 5]");
    for (int t = 0; t < n; ++t) {
        const int rc = wgrad_validate(&ds[t]);
        if (rc != ISR_OK) return rc;
        if (ds[t].g_sub2 || ds[t].x_sub2 || ds[t].taps || ds[t].n != ds[0].n || ds[t].ha != ds[0].ha ||
            ds[t].wa != ds[0].wa)
            return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3 group: member %d is not a plain 3x3 conv on the first "
                        "member's grid", t);
    }
    return ISR_OK;
}

size_t isr_wgrad3x3_group_workspace_bytes(const isr_wgrad_desc* descs, int32_t n) {
    if (wgrad_group_validate(descs, n) != ISR_OK) return 0;
    return isr::wgrad3x3_group_workspace_bytes(descs, n, 0);
}

int isr_wgrad3x3_group_variant(const isr_wgrad_desc* descs, int32_t n, int32_t variant, void* workspace,
                               size_t ws_bytes, isr_stream_t s) {
    int rc = wgrad_group_validate(descs, n);
    if (rc != ISR_OK) return rc;
    if (!workspace) return fail(ISR_ERR_BAD_DESC, "wgrad3x3 group: null workspace");
    if (variant != 0 && variant != 1) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3 group: no variant %d", variant);
    rc = isr::wgrad3x3_group_dispatch(descs, n, workspace, ws_bytes, (hipStream_t)s, variant);
    if (rc == -3) return fail(ISR_ERR_BAD_DESC, "wgrad3x3 group: workspace of %zu bytes is smaller than %zu", ws_bytes,
                              isr::wgrad3x3_group_workspace_bytes(descs, n, variant));
    if (rc == -2) return fail(ISR_ERR_UNSUPPORTED, "wgrad3x3 group: a member's cout / cin / ha does not fit the tile");
    return launched(rc, "wgrad3x3 group");
}

int isr_wgrad3x3_group(const isr_wgrad_desc* descs, int32_t n, void* workspace, size_t ws_bytes, isr_stream_t s) {
    return isr_wgrad3x3_group_variant(descs, n, 0, workspace, ws_bytes, s);
}

int isr_wgrad3x3_partials(const isr_wgrad_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s) {
    return wgrad3x3_parts(d, 0, workspace, ws_bytes, s, 1);
}

int isr_wgrad3x3_reduce(const isr_wgrad_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s) {
    return wgrad3x3_parts(d, 0, workspace, ws_bytes, s, 2);
}

size_t isr_wgrad3x3_variant_workspace_bytes(const isr_wgrad_desc* d, int32_t variant) {
    if (wgrad_validate(d) != ISR_OK || !wgrad_variant_built(variant)) return 0;
    return isr::wgrad3x3_workspace_bytes(d, variant);
}

static int wgrad9_validate(const isr_wgrad9_desc* d) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "wgrad9x9: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0) return fail(ISR_ERR_BAD_DESC, "wgrad9x9: empty problem");
    if (d->ha % ISR_TILE_H || d->wa % ISR_TILE_W || d->ha < d->h || d->wa < d->w)
        return fail(ISR_ERR_BAD_DESC, "wgrad9x9: bad computed region %dx%d for %dx%d", d->ha, d->wa, d->h, d->w);
    if (!d->p || !d->dw) return fail(ISR_ERR_BAD_DESC, "wgrad9x9: null p / dw");
    if (d->splits < 0) return fail(ISR_ERR_BAD_DESC, "wgrad9x9: negative split count");
    if (!view_ok(d->q, d->ha, d->wa, d->head ? 0 : 4, 64, "wgrad9x9.q", 1)) return ISR_ERR_BAD_DESC;
    return ISR_OK;
}

size_t isr_wgrad9x9_workspace_bytes(const isr_wgrad9_desc* d) {
    if (wgrad9_validate(d) != ISR_OK) return 0;
    return isr::wgrad9x9_workspace_bytes(d);
}

int isr_wgrad9x9(const isr_wgrad9_desc* d, void* workspace, size_t ws_bytes, isr_stream_t s) {
    int rc = wgrad9_validate(d);
    if (rc != ISR_OK) return rc;
    if (!workspace) return fail(ISR_ERR_BAD_DESC, "wgrad9x9: null workspace");
    rc = isr::wgrad9x9_dispatch(d, workspace, ws_bytes, (hipStream_t)s);
    if (rc == -3) return fail(ISR_ERR_BAD_DESC, "wgrad9x9: workspace too small");
    return launched(rc, "wgrad9x9");
}

int isr_ew_combine(const isr_ew_desc* d, isr_stream_t s) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "ew_combine: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0 || d->c % 16)
        return fail(ISR_ERR_BAD_DESC, "ew_combine: bad problem n=%d h=%d w=%d c=%d", d->n, d->h, d->w, d->c);
    if (d->ha < d->h || d->wa < d->w) return fail(ISR_ERR_BAD_DESC, "ew_combine: computed region smaller than valid");
    if (!view_ok(d->y, d->ha, d->wa, 0, d->c, "ew.y", 1) || !view_ok(d->a, d->ha, d->wa, 0, d->c, "ew.a", 1))
        return ISR_ERR_BAD_DESC;
    if (d->b.data && !view_ok(d->b, d->ha, d->wa, 0, d->c, "ew.b", 1)) return ISR_ERR_BAD_DESC;
    if (d->m.data && !view_ok(d->m, d->ha, d->wa, 0, d->c, "ew.m", 1)) return ISR_ERR_BAD_DESC;
    return launched(isr::ew_combine_dispatch(d, (hipStream_t)s), "ew_combine");
}

int isr_sr_transform(const isr_sr_transform_desc* d, isr_stream_t s) {
    if (!d || !d->crops || !d->hr || !d->lr) return fail(ISR_ERR_BAD_DESC, "sr_transform: null descriptor / buffer");
    if (d->scale < 2 || d->scale > 4) return fail(ISR_ERR_UNSUPPORTED, "sr_transform: scale %d not in {2, 3, 4}", d->scale);
    if (d->n <= 0 || d->t <= 0 || d->t % d->scale || (long long)d->n * 3 * d->t * d->t >= (1ll << 31))
        return fail(ISR_ERR_BAD_DESC, "sr_transform: bad batch n=%d t=%d scale=%d", d->n, d->t, d->scale);
    for (int c = 0; c < 3; ++c)
        if (!(d->std[c] != 0.f)) return fail(ISR_ERR_BAD_DESC, "sr_transform: std[%d] is zero", c);
    return launched(isr::sr_transform_dispatch(d, (hipStream_t)s), "sr_transform");
}

int isr_pixel_shuffle2(const isr_ew_desc* d, isr_stream_t s) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "pixel_shuffle2: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0 || d->c % 16)
        return fail(ISR_ERR_BAD_DESC, "pixel_shuffle2: bad problem n=%d h=%d w=%d c=%d", d->n, d->h, d->w, d->c);
    if (d->h % 2 || d->w % 2) return fail(ISR_ERR_BAD_DESC, "pixel_shuffle2: output %dx%d must be even", d->h, d->w);
    if (d->ha < d->h || d->wa < d->w || d->ha % 2 || d->wa % 2)
        return fail(ISR_ERR_BAD_DESC, "pixel_shuffle2: computed region %dx%d must be even and cover %dx%d", d->ha, d->wa,
                    d->h, d->w);
    if (d->b.data || d->m.data) return fail(ISR_ERR_UNSUPPORTED, "pixel_shuffle2: takes no b / m operand");
    if (!view_ok(d->y, d->ha, d->wa, 0, d->c, "pixel_shuffle2.y", 1) ||
        !view_ok(d->a, d->ha / 2, d->wa / 2, 0, 4 * d->c, "pixel_shuffle2.a", 1))
        return ISR_ERR_BAD_DESC;
    return launched(isr::pixel_shuffle2_dispatch(d, (hipStream_t)s), "pixel_shuffle2");
}

int isr_pixel_unshuffle2(const isr_ew_desc* d, isr_stream_t s) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "pixel_unshuffle2: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0 || d->c % 64)
        return fail(ISR_ERR_BAD_DESC, "pixel_unshuffle2: bad problem n=%d h=%d w=%d c=%d (c %% 64 == 0)", d->n, d->h,
                    d->w, d->c);
    if (d->ha < d->h || d->wa < d->w) return fail(ISR_ERR_BAD_DESC, "pixel_unshuffle2: computed region smaller than valid");
    if (d->b.data) return fail(ISR_ERR_UNSUPPORTED, "pixel_unshuffle2: takes no b operand");
    if (!view_ok(d->y, d->ha, d->wa, 0, d->c, "pixel_unshuffle2.y", 1) ||
        !view_ok(d->a, 2 * d->ha, 2 * d->wa, 0, d->c / 4, "pixel_unshuffle2.a", 1))
        return ISR_ERR_BAD_DESC;
    if (d->m.data && !view_ok(d->m, 2 * d->ha, 2 * d->wa, 0, d->c / 4, "pixel_unshuffle2.m", 1)) return ISR_ERR_BAD_DESC;
    return launched(isr::pixel_unshuffle2_dispatch(d, (hipStream_t)s), "pixel_unshuffle2");
}

static int convert_validate(const isr_convert_desc* d, const char* who) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "%s: null descriptor", who);
    if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0) return fail(ISR_ERR_BAD_DESC, "%s: empty problem", who);
    if (d->ha < d->h || d->wa < d->w) return fail(ISR_ERR_BAD_DESC, "%s: computed region smaller than valid", who);
    if (!d->nchw) return fail(ISR_ERR_BAD_DESC, "%s: null nchw pointer", who);
    if (!view_ok(d->v, d->ha, d->wa, 0, (d->c + 15) / 16 * 16, who, 1)) return ISR_ERR_BAD_DESC;
    if (d->m.data && !view_ok(d->m, d->ha, d->wa, 0, (d->c + 15) / 16 * 16, who, 1)) return ISR_ERR_BAD_DESC;
    return ISR_OK;
}

int isr_nchw_to_blocked(const isr_convert_desc* d, isr_stream_t s) {
    int rc = convert_validate(d, "nchw_to_blocked");
    if (rc != ISR_OK) return rc;
    return launched(isr::nchw_to_blocked_dispatch(d, (hipStream_t)s), "nchw_to_blocked");
}

int isr_blocked_to_nchw(const isr_convert_desc* d, isr_stream_t s) {
    int rc = convert_validate(d, "blocked_to_nchw");
    if (rc != ISR_OK) return rc;
    return launched(isr::blocked_to_nchw_dispatch(d, (hipStream_t)s), "blocked_to_nchw");
}

static int pool_validate(const isr_pool_desc* d, int bwd) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "maxpool2: null descriptor");
    if (d->n <= 0 || d->h < 2 || d->w < 2 || d->c <= 0 || d->c % 16)
        return fail(ISR_ERR_BAD_DESC, "maxpool2: bad problem n=%d h=%d w=%d c=%d", d->n, d->h, d->w, d->c);
    if (d->hao < d->h / 2 || d->wao < d->w / 2) return fail(ISR_ERR_BAD_DESC, "maxpool2: output region too small");
    if (!view_ok(d->x, 2 * d->hao, 2 * d->wao, 0, d->c, "maxpool2.x", 1)) return ISR_ERR_BAD_DESC;
    if (!view_ok(d->y, d->hao, d->wao, 0, d->c, "maxpool2.y", 1)) return ISR_ERR_BAD_DESC;
    if (bwd && !view_ok(d->g, 2 * d->hao, 2 * d->wao, 0, d->c, "maxpool2.g", 1)) return ISR_ERR_BAD_DESC;
    return ISR_OK;
}

int isr_maxpool2_fwd(const isr_pool_desc* d, isr_stream_t s) {
    int rc = pool_validate(d, 0);
    if (rc != ISR_OK) return rc;
    return launched(isr::maxpool2_dispatch(d, 0, (hipStream_t)s), "maxpool2_fwd");
}

int isr_maxpool2_bwd(const isr_pool_desc* d, isr_stream_t s) {
    int rc = pool_validate(d, 1);
    if (rc != ISR_OK) return rc;
    return launched(isr::maxpool2_dispatch(d, 1, (hipStream_t)s), "maxpool2_bwd");
}

static int bn_validate(const isr_bn_desc* d, int op) {
    if (!d) return fail(ISR_ERR_BAD_DESC, "bn: null descriptor");
    if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0 || d->c % 16 || d->c > 1024)
        return fail(ISR_ERR_BAD_DESC, "bn: bad problem n=%d h=%d w=%d c=%d (c %% 16 == 0, c <= 1024)", d->n, d->h,
                    d->w, d->c);
    if (d->ha < d->h || d->wa < d->w) return fail(ISR_ERR_BAD_DESC, "bn: computed region smaller than valid");
    if (!d->acc || !d->save) return fail(ISR_ERR_BAD_DESC, "bn: null acc / save");
    if (op != 1 && !view_ok(d->z, d->ha, d->wa, 0, d->c, "bn.z", 1)) return ISR_ERR_BAD_DESC;
    if ((op == 2 || op >= 3) && !view_ok(d->y, d->ha, d->wa, 0, d->c, "bn.y", 1)) return ISR_ERR_BAD_DESC;
    if (op == 2 && d->r1.data && !view_ok(d->r1, d->ha, d->wa, 0, d->c, "bn.r1", 1)) return ISR_ERR_BAD_DESC;
    if (op == 2 && d->r2.data && !view_ok(d->r2, d->ha, d->wa, 0, d->c, "bn.r2", 1)) return ISR_ERR_BAD_DESC;
    if (op == 4 && d->dz.data && !view_ok(d->dz, d->ha, d->wa, 0, d->c, "bn.dz", 1)) return ISR_ERR_BAD_DESC;
    if ((op == 2 || op == 4) && (!d->gamma || (op == 2 && !d->beta)))
        return fail(ISR_ERR_BAD_DESC, "bn: null gamma / beta");
    if (op == 1 && (!d->running_mean) != (!d->running_var)) return fail(ISR_ERR_BAD_DESC, "bn: running stats pair");
    return ISR_OK;
}

static int bn_run(const isr_bn_desc* d, int op, isr_stream_t s, const char* what) {
    int rc = bn_validate(d, op);
    if (rc != ISR_OK) return rc;
    return launched(isr::bn_dispatch(d, op, (hipStream_t)s), what);
}

int isr_bn_stats(const isr_bn_desc* d, isr_stream_t s) { return bn_run(d, 0, s, "bn_stats"); }
int isr_bn_finalize(const isr_bn_desc* d, isr_stream_t s) { return bn_run(d, 1, s, "bn_finalize"); }
int isr_bn_apply(const isr_bn_desc* d, isr_stream_t s) { return bn_run(d, 2, s, "bn_apply"); }
int isr_bn_bwd_reduce(const isr_bn_desc* d, isr_stream_t s) { return bn_run(d, 3, s, "bn_bwd_reduce"); }
int isr_bn_bwd_apply(const isr_bn_desc* d, isr_stream_t s) { return bn_run(d, 4, s, "bn_bwd_apply"); }

}  // extern "C"
