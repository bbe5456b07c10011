"""Inference engine for the RRDB generators on libisr (MI355X).

Executes ResNet / EResNet (utils/models.py:592-650) — optionally wrapped as
the uint8 `Model` (:723-739) — entirely through the HIP kernels:

  head9x9   conv0 (+Normalize for uint8 input)       → feat, X[0:64]
  16 x RRDB, each 3 x RDB on rotating dense buffers X → Y → Z → X:
    conv3x3 growth k=0..3  src[0:64+32k] → src[64+32k : 96+32k]     (torch.cat eliminated)
    conv3x3 final          src[0:192] → dst[0:64],  v*0.2 + src[0:64]
                           (third RDB: ((v*0.2 + Z) * 0.2 + X) in place = RRDB residual)
  conv3x3 conv1            X[0:64] → feat (in place), v + feat    (trunk residual)
  conv3x3 scaler x S       64 → 256, PixelShuffle(2) + LeakyReLU on store
  tail9x9 conv2 + tanh     → NCHW fp32 (or uint8 = TanhToArrayImage)

Activations are channel-blocked fp16 (the default storage of this inference path; bf16 with
pack_generator(f16=False)) with a zero border (ops.ActBuffer); the dense
buffers keep the 192-channel concat resident so no concat is ever copied.
BatchNorm is folded into the conv (fuse_conv_and_bn, :366-406) at pack time.
"""
from __future__ import annotations

import ctypes
import warnings
from dataclasses import dataclass, field

import torch

from . import ops
from .ops import ActBuffer

LEAKY_DEFAULT = 0.01


def _fold(sd: dict, prefix: str, device) -> tuple[torch.Tensor, torch.Tensor]:
    """(W, b) fp32 of Conv / ConvWithoutBN `prefix`, BN folded as fuse_conv_and_bn does."""
    w = sd[f"{prefix}.conv.weight"].detach().to(device=device, dtype=torch.float32)
    b = sd.get(f"{prefix}.conv.bias")
    b = torch.zeros(w.shape[0], device=device) if b is None else b.detach().to(device=device, dtype=torch.float32)
    if f"{prefix}.bn.weight" in sd:
        g = sd[f"{prefix}.bn.weight"].detach().to(device, torch.float32)
        beta = sd[f"{prefix}.bn.bias"].detach().to(device, torch.float32)
        mu = sd[f"{prefix}.bn.running_mean"].detach().to(device, torch.float32)
        var = sd[f"{prefix}.bn.running_var"].detach().to(device, torch.float32)
        eps = 1e-5
        s = g / torch.sqrt(eps + var)
        w = w * s.view(-1, 1, 1, 1)
        b = s * b + (beta - g * mu / torch.sqrt(var + eps))
    return w, b.contiguous()


@dataclass
class PackedConv:
    w: torch.Tensor  # packed bf16 or fp16 (the storage type of the launches that use it)
    b: torch.Tensor  # fp32 bias
    cin: int
    cout: int


@dataclass
class GeneratorWeights:
    head: PackedConv
    rdb: list[list[list[PackedConv]]]  # [block][rdb 0..2][conv 0..4]
    conv1: PackedConv
    scalers: list[PackedConv]
    tail: PackedConv
    conv0_slope: float
    add_rate: float
    buffers: dict = field(default_factory=dict)

    @property
    def dtype(self) -> torch.dtype:
        """Storage type of the packed weights, hence of every activation buffer of a plan."""
        return self.head.w.dtype


def _pack3(sd, prefix, device, f16: bool = False) -> PackedConv:
    w, b = _fold(sd, prefix, device)
    return PackedConv(ops.pack_conv3x3(w, f16=f16), b, w.shape[1], w.shape[0])


def count_blocks(sd: dict, prefix: str = "") -> int:
    p = f"{prefix}residual."
    return len({int(k[len(p):].split(".")[0]) for k in sd if k.startswith(p)})


def count_scalers(sd: dict, prefix: str = "") -> int:
    p = f"{prefix}scaler."
    return len({int(k[len(p):].split(".")[0]) for k in sd if k.startswith(p)})


def pack_generator(sd: dict, *, enchant: bool, add_rate: float = 0.2, prefix: str = "",
                   device="cuda", f16: bool = True) -> GeneratorWeights:
    """Pack a ResNet/EResNet state_dict (reference key schema, fused or not).

    `f16` (default): fp16 weights and activations — the inference path's storage type, 3 more
    mantissa bits than bf16 at the same MFMA rate and bytes (x2 generator vs the fp32 oracle:
    78.9 dB against 59.7 dB in bf16); f16=False keeps bf16 storage."""
    p = prefix
    w0, b0 = _fold(sd, f"{p}conv0", device)
    head = PackedConv(ops.pack_head9x9(w0, f16=f16), b0, w0.shape[1], w0.shape[0])
    nb = count_blocks(sd, p)
    rdb = [[[_pack3(sd, f"{p}residual.{i}.net.{r}.{c}", device, f16)
             for c in ("conv0", "conv1", "conv2", "conv3", "conv")] for r in range(3)] for i in range(nb)]
    conv1 = _pack3(sd, f"{p}conv1", device, f16)
    scalers = [_pack3(sd, f"{p}scaler.{s}.net.0", device, f16) for s in range(count_scalers(sd, p))]
    w2, b2 = _fold(sd, f"{p}conv2", device)
    tail = PackedConv(ops.pack_tail9x9(w2, f16=f16), b2, w2.shape[1], w2.shape[0])
    return GeneratorWeights(head, rdb, conv1, scalers, tail, LEAKY_DEFAULT if enchant else 0.2, add_rate)


class GeneratorBuffers:
    """Activation buffers for one input geometry, allocated once and reused."""

    def __init__(self, n: int, h: int, w: int, n_scalers: int, device, dtype: torch.dtype = torch.bfloat16):
        self.feat = ActBuffer.alloc(n, h, w, 64, 1, device, dtype=dtype)
        self.dense = [ActBuffer.alloc(n, h, w, 192, 1, device, dtype=dtype) for _ in range(3)]
        self.up = []
        hh, ww = h, w
        ha, wa = self.feat.ha, self.feat.wa
        for s in range(n_scalers):
            hh, ww, ha, wa = 2 * hh, 2 * ww, 2 * ha, 2 * wa
            pad = 4 if s == n_scalers - 1 else 1
            self.up.append(ActBuffer.alloc(n, hh, ww, 64, pad, device, ha=ha, wa=wa, dtype=dtype))


def rdb_forward(convs: list[PackedConv], src: ActBuffer, dst: ActBuffer, add_rate: float, *,
                r2: ActBuffer | None = None, s2: float = 1.0, slope: float = LEAKY_DEFAULT) -> None:
    """RDB.forward (utils/models.py:265-271) on a 192-channel dense buffer.

    src[0:64] holds the block input; growth conv k appends channels
    [64+32k, 96+32k) in place (the torch.cat chain), the final conv writes
    dst[0:64] = conv*add_rate + src[0:64] (then *s2 + r2 when r2 is given —
    the enclosing RRDB's residual, utils/models.py:317)."""
    for k in range(4):
        pc = convs[k]
        ops.conv3x3(src, pc.cin, pc.w, pc.b, pc.cout, src, y_coff=pc.cin, slope=slope)
    pc = convs[4]
    ops.conv3x3(src, pc.cin, pc.w, pc.b, pc.cout, dst, slope=1.0, r1=src, s1=add_rate, r2=r2, s2=s2)


def rrdb_forward(blk, X: ActBuffer, Y: ActBuffer, Z: ActBuffer, add_rate: float, *,
                 slope: float = LEAKY_DEFAULT) -> None:
    """RRDB.forward (utils/models.py:316-317): X → Y → Z → X[0:64] (in place), where
    the last RDB's epilogue adds the RRDB residual X[0:64] at the same pixel."""
    rdb_forward(blk[0], X, Y, add_rate, slope=slope)
    rdb_forward(blk[1], Y, Z, add_rate, slope=slope)
    rdb_forward(blk[2], Z, X, add_rate, r2=X, s2=add_rate, slope=slope)


class GeneratorPlan:
    """Pre-built launch list of one generator forward for a fixed geometry.

    Building ctypes descriptors costs tens of microseconds each in Python;
    a forward has ~245 launches, so descriptors are built once per geometry
    and only the input / output pointers are patched per call.  Each entry
    carries a tag (kind, cin, cout) so callers can bracket the launches of
    one kernel shape with HIP events (bench.py).
    """

    def __init__(self, gw: GeneratorWeights, n: int, h: int, w: int, device, x_u8: bool, out_u8: bool,
                 mean, std, variants: dict | None = None, chain: bool | None = None,
                 chain_acquire: bool | None = None):
        """`variants` (tuning only) maps ("conv3x3", cin, cout) or ("conv3x3", "*", cout)
        to an isr_conv3x3_fwd_variant id; unlisted convs use the production kernel.
        `chain` (default CHAIN_DEFAULT): the RRDB trunk as one persistent isr_conv_chain launch."""
        if chain is None:
            chain = CHAIN_DEFAULT
        if chain_acquire is None:
            chain_acquire = CHAIN_ACQUIRE
        self.key = (n, h, w, str(device), x_u8, out_u8, tuple(mean), tuple(std))
        # the descriptors hold raw pointers into gw's packed weights: the plan keeps gw alive (a plan
        # that outlived its weights read whatever reused that memory — found by tools/ab_storage.py,
        # whose bf16 plan's weights were freed and refilled by the fp16 packs built after it)
        self.gw = gw
        bufs = GeneratorBuffers(n, h, w, len(gw.scalers), device, gw.dtype)
        self.bufs = bufs
        feat = bufs.feat
        X, Y, Z = bufs.dense
        lib = ops._lib.load()
        conv, head, tail = lib.isr_conv3x3_fwd, lib.isr_head9x9_fwd, lib.isr_tail9x9_fwd
        dummy_x = torch.empty((n, 3, h, w), dtype=torch.uint8 if x_u8 else torch.float32, device=device)
        cur_h, cur_w = h * 2 ** len(gw.scalers), w * 2 ** len(gw.scalers)
        self.out_shape = (n, 3, cur_h, cur_w)
        self.out_dtype = torch.uint8 if out_u8 else torch.float32
        dummy_out = torch.empty(self.out_shape, dtype=self.out_dtype, device=device)
        self.head_desc = ops.head9x9_desc(dummy_x, gw.head.w, gw.head.b, feat, slope=gw.conv0_slope, y2=X,
                                          mean=mean, std=std)
        L = [(head, self.head_desc, ("head9x9", 3, 64), None)]
        self._conv_variant = lib.isr_conv3x3_fwd_variant

        def c3(src, pc, dst, **kw):
            tag = ("conv3x3", pc.cin, pc.cout)
            v = (variants or {}).get(tag, (variants or {}).get(("conv3x3", "*", pc.cout)))
            L.append((conv, ops.conv3x3_desc(src, pc.cin, pc.w, pc.b, pc.cout, dst, **kw), tag, v))

        ar = gw.add_rate
        trunk0 = len(L)
        for blk in gw.rdb:
            for r, (src, dst) in enumerate(((X, Y), (Y, Z), (Z, X))):
                for k in range(4):
                    c3(src, blk[r][k], src, y_coff=blk[r][k].cin, slope=LEAKY_DEFAULT)
                extra = dict(r2=X, s2=ar) if r == 2 else {}
                c3(src, blk[r][4], dst, slope=1.0, r1=src, s1=ar, **extra)
        self.chain = None
        if chain and gw.rdb and all(e[3] is None for e in L[trunk0:]):  # variants may only touch other layers
            # the whole RRDB trunk as ONE persistent launch (isr_conv_chain): tile-level
            # dependencies instead of 240 kernel boundaries
            try:
                self.chain = ConvChain([d for _, d, _, _ in L[trunk0:]], X, device, acquire=chain_acquire)
            except ValueError as e:  # e.g. buffers beyond the 2 GiB descriptor window: per-conv launches
                warnings.warn(f"RRDB trunk on 240 per-conv launches instead of the persistent trunk kernel: {e}",
                              stacklevel=2)
                self.chain = None
            if self.chain is not None:
                L[trunk0:] = [(self.chain.fn, self.chain.desc, ("chain", len(L) - trunk0), None)]
        c3(X, gw.conv1, feat, slope=1.0, r1=feat, s1=1.0)
        cur = feat
        for s, pc in enumerate(gw.scalers):
            c3(cur, pc, bufs.up[s], slope=LEAKY_DEFAULT, shuffle=2)
            cur = bufs.up[s]
        self.tail_desc = ops.tail9x9_desc(cur, gw.tail.w, gw.tail.b, dummy_out)
        L.append((tail, self.tail_desc, ("tail9x9", 64, 3), None))
        self.launches = L
        self._keep = (dummy_x, dummy_out)

    def bind(self, x: torch.Tensor, out: torch.Tensor) -> None:
        if tuple(out.shape) != self.out_shape or out.dtype != self.out_dtype or not out.is_contiguous():
            raise ValueError("GeneratorPlan.run: output tensor does not match the plan")
        if not x.is_contiguous():
            raise ValueError("GeneratorPlan.run: input must be contiguous NCHW")
        self.head_desc.x = x.data_ptr()
        self.tail_desc.y = out.data_ptr()

    def run(self, x: torch.Tensor, out: torch.Tensor, around=None) -> torch.Tensor:
        """Launch the forward on the current stream.  `around(tag)` may return
        (start_event, end_event) to bracket that launch."""
        self.bind(x, out)
        stream = ops._stream()
        byref = ctypes.byref
        cv = self._conv_variant
        for fn, d, tag, var in self.launches:
            ev = around(tag) if around is not None else None
            if ev is not None:
                ev[0].record()
            rc = fn(byref(d), stream) if var is None else cv(byref(d), var, stream)
            if rc != 0:
                ops.check(rc, f"{tag[0]} launch")
            if ev is not None:
                ev[1].record()
        if self.chain is not None and not torch.cuda.is_current_stream_capturing():
            self.chain.poll()
        return out

    @property
    def chains(self) -> list:
        return [self.chain] if self.chain is not None else []

    def verify(self) -> None:
        """Blocking give-up check of every forward queued so far (one-shot consumers call it
        before handing results out: the tiler's canvas, a training epoch end)."""
        for c in self.chains:
            c.verify()


class ChainFailed(RuntimeError):
    """A persistent-chain dependency wait gave up (a neighbour tile never published: the
    launch was not fully resident) — that launch's outputs are invalid."""


class ConvChain:
    """Device-side layer table + state for isr_conv_chain over a run of RDB convs
    (growth convs: kind 0; 192→64 final convs: kind 1) sharing one tile grid."""

    def __init__(self, descs, grid: ActBuffer, device, acquire: bool = False, variant: int | None = None,
                 state: torch.Tensor | None = None):
        """`state`: share another chain's state words (chains launched one after another on one
        stream: generations and progress words are serial, and one give-up count guards both)."""
        lib = ops._lib.load()
        kinds = []
        g = descs[0].x
        for d in descs:
            ops.check(lib.isr_conv3x3_check(ctypes.byref(d)), "chain layer")
            if d.cout == 32:
                # kind 2: the training backward's RDB gather conv (LeakyReLU' mask epilogue)
                kinds.append(2 if d.m.data else 0)
            elif d.cin == 192 and d.cout == 64:
                kinds.append(1)
            else:
                raise ValueError(f"conv chain: unsupported layer {d.cin}->{d.cout}")
            if d.x_sub2 or d.taps or d.shuffle != 1 or d.y2.data:
                raise ValueError("conv chain: plain 3x3 layers only")
            if d.m.data and (d.m_c0 != 0 or d.slope != 1.0 or d.r1.data or d.r2.data or d.s1 != 1.0 or d.s2 != 1.0
                             or (d.m.hp, d.m.wp, d.m.cs, d.m.pad) != (g.hp, g.wp, g.cs, g.pad)):
                raise ValueError("conv chain: a masked layer is a plain 32-cout conv whose every channel is "
                                 "masked by a buffer of the chain's geometry")
            if (d.n, d.ha, d.wa) != (grid.n, grid.ha, grid.wa):
                raise ValueError("conv chain: every layer must share the tile grid")
            # the trunk kernel's layer records (trunk.hip) share one view geometry and fold r1
            views = [d.x, d.y] + ([d.r2] if d.r2.data else [])
            if any((v.hp, v.wp, v.cs, v.pad) != (g.hp, g.wp, g.cs, g.pad) for v in views) or not d.bias:
                raise ValueError("conv chain: every layer must share one buffer geometry and carry a bias")
            if d.r1.data and not (d.r1.data == d.x.data and d.r1.coff == d.x.coff and d.r1_cn == 0
                                  and d.slope == 1.0 and _storage_exact(1.0 / d.s1, d.f16)):
                raise ValueError("conv chain: r1 must be the layer's own input (identity activation, "
                                 "1/s1 exact in the storage type)")
            if d.r2.data and not d.r1.data:
                raise ValueError("conv chain: r2 without r1")
        f16 = {d.f16 for d in descs}
        if len(f16) != 1 or f16 != {grid.f16}:
            raise ValueError("conv chain: every layer must share the grid's storage type")
        if grid.t.shape[2] * grid.t.shape[3] * 32 >= 2 ** 31:  # the trunk kernel's buffer resources span one 16-channel plane
            raise ValueError("conv chain: a 16-channel activation plane must stay below 2 GiB (buffer-descriptor "
                             "window)")
        self.variant = CHAIN_VARIANT if variant is None else variant
        if grid.f16 and (2 in kinds or self.variant != 0):
            raise ValueError("conv chain: fp16 storage runs the production trunk form (forward layers) only")
        if self.variant in (3, 4) and grid.ha % 32:
            raise ValueError(f"conv chain: variant {self.variant} (32x32 trunk tiles) needs the padded height "
                             "a multiple of 32")
        if self.variant == 1 and grid.t.numel() * grid.t.element_size() >= 2 ** 31:
            # the round-2 kernel's hand-off loads / stores address a whole buffer through one
            # descriptor with 32-bit offsets (isr_common.h rsrc_of)
            raise ValueError("conv chain: variant 1 (the round-2 kernel) needs every activation buffer below "
                             "2 GiB")
        if 2 in kinds and self.variant in (1, 4):
            raise ValueError(f"conv chain: variant {self.variant} has no masked (kind 2) layers")
        if self.variant == 4 and any(d.cin % 32 or (k == 1 and (not d.r1.data or d.cin < 96))
                                     for d, k in zip(descs, kinds)):
            raise ValueError("conv chain: variant 4 pairs 16-channel chunks (cin % 32 == 0) and needs every "
                             "64-cout layer to fold its residual r1 (cin >= 96)")
        raw = b"".join(bytes(d) for d in descs)
        self._table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self._kinds = torch.tensor(kinds, dtype=torch.int32, device=device)
        words = lib.isr_conv_chain_state_words(grid.n, grid.ha, grid.wa)
        if state is not None:
            if state.numel() < words or state.dtype != torch.int32:
                raise ValueError("conv chain: shared state too small")
            self.state = state
        else:
            self.state = torch.zeros(words, dtype=torch.int32, device=device)
        self.desc = ops._lib.IsrChainDesc(self._table.data_ptr(), self._kinds.data_ptr(), len(descs), grid.n,
                                          grid.ha, grid.wa, self.state.data_ptr(), int(acquire), grid.f16)
        self.nl = len(descs)
        if self.variant == 0:
            self.fn = lib.isr_conv_chain
        else:
            fv, var = lib.isr_conv_chain_variant, self.variant
            self.fn = lambda d, s: fv(d, var, s)

    def failed(self) -> bool:
        """True when a dependency wait gave up in the last launch (results invalid).  Synchronous
        (tests and tools)."""
        gen, fail = self.state[:2].tolist()
        return gen != 0 and fail == gen

    # ---- product-path checks.  state[2] counts give-ups over every launch and is never reset,
    # so a snapshot taken after ANY later launch still shows an earlier failure (the video
    # pipeline's double-buffered slots can read a newer snapshot than the batch they check).
    def snapshot(self, dst: torch.Tensor) -> None:
        """Enqueue (current stream) an async copy of the give-up count into pinned `dst` (int32[1])."""
        dst.copy_(self.state[2:3], non_blocking=True)

    @property
    def guard_ptr(self) -> int:
        """Device address of state words [2, 3] (the sticky give-up count, the count the host has
        accepted): the guard of optim's HIP Adam / EMA updates (isr_mt_adam_guarded)."""
        return self.state.data_ptr() + 8

    def check_count(self, count: int) -> None:
        """Raise ChainFailed when `count` (a snapshot) shows a give-up not yet reported; the
        reported count becomes the accepted one (state[3]), so guarded optimiser updates of
        launches after it run again once the caller has handled the error."""
        seen = getattr(self, "_fails_seen", 0)
        if count != seen:
            self._fails_seen = count
            self.state[3:4].fill_(count)
            raise ChainFailed("conv chain: a dependency wait gave up (launch not fully resident); "
                              "outputs of that forward are invalid")

    def poll(self) -> None:
        """Lagged, non-blocking check after every eager forward: raises ChainFailed when the
        snapshot queued after an earlier launch shows a give-up; then queues a snapshot after the
        launch just issued.  Never synchronises (an unfinished copy is checked on a later call)."""
        ev = getattr(self, "_poll_ev", None)
        if ev is not None and ev.query():
            self.check_count(int(self._poll_host[0]))
        elif ev is not None:
            return  # the previous copy has not landed yet: keep it, check it later
        if getattr(self, "_poll_host", None) is None:
            self._poll_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._poll_ev = torch.cuda.Event()
        self.snapshot(self._poll_host)
        self._poll_ev.record()

    def verify(self) -> None:
        """Blocking check of every launch queued so far on the current stream (waits for them,
        not for the whole device): raises ChainFailed on a give-up."""
        if getattr(self, "_verify_host", None) is None:
            self._verify_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._verify_ev = torch.cuda.Event()
        self.snapshot(self._verify_host)
        self._verify_ev.record()
        self._verify_ev.synchronize()
        self.check_count(int(self._verify_host[0]))


class SplitGeneratorPlan:
    """The batch split into `splits` equal sub-batches, each with its own buffers
    and launch list on its own HIP stream; launches are issued interleaved
    (layer i of every sub-batch, then layer i+1).  Sub-batch k > 0 starts
    `stagger_us * k` later, so that one sub-batch's epilogue (HBM-bound) runs
    beside another's main loop (MFMA-bound) on the same CUs."""

    def __init__(self, gw: GeneratorWeights, n: int, h: int, w: int, device, x_u8: bool, out_u8: bool,
                 mean, std, splits: int = 2, stagger_us: float = 0.0, variants: dict | None = None,
                 chain: bool | None = None):
        if n % splits:
            raise ValueError(f"batch {n} does not split into {splits} equal sub-batches")
        self.m = n // splits
        self.key = (n, h, w, str(device), x_u8, out_u8, tuple(mean), tuple(std), splits, stagger_us)
        # no persistent chain in the sub-plans: their launches run concurrently on separate
        # streams, and two grids that each fill the device cannot all be resident (waits would
        # give up); the split plan is the per-conv form only
        self.subs = [GeneratorPlan(gw, self.m, h, w, device, x_u8, out_u8, mean, std, variants=variants,
                                   chain=False) for _ in range(splits)]
        self.out_shape = (n,) + self.subs[0].out_shape[1:]
        self.out_dtype = self.subs[0].out_dtype
        self.streams = [torch.cuda.Stream(device) for _ in range(splits)]
        self._sp = [ctypes.c_void_p(s.cuda_stream) for s in self.streams]
        self.stagger_cycles = int(stagger_us * _sleep_cycles_per_us()) if stagger_us > 0 else 0

    def run(self, x: torch.Tensor, out: torch.Tensor, around=None) -> torch.Tensor:
        if tuple(out.shape) != self.out_shape or out.dtype != self.out_dtype or not out.is_contiguous():
            raise ValueError("SplitGeneratorPlan.run: output tensor does not match the plan")
        m = self.m
        for k, p in enumerate(self.subs):
            p.bind(x[k * m:(k + 1) * m], out[k * m:(k + 1) * m])
        cur = torch.cuda.current_stream()
        for k, s in enumerate(self.streams):
            s.wait_stream(cur)
            if k and self.stagger_cycles:
                with torch.cuda.stream(s):
                    torch.cuda._sleep(self.stagger_cycles * k)
        byref = ctypes.byref
        cv = self.subs[0]._conv_variant
        lists = [p.launches for p in self.subs]
        for i in range(len(lists[0])):
            for k, L in enumerate(lists):
                fn, d, tag, var = L[i]
                rc = fn(byref(d), self._sp[k]) if var is None else cv(byref(d), var, self._sp[k])
                if rc != 0:
                    ops.check(rc, f"{tag[0]} launch")
        for s in self.streams:
            cur.wait_stream(s)
        return out

    chains: list = []

    def verify(self) -> None:
        pass


_SLEEP_CAL: list[float] = []


def _sleep_cycles_per_us() -> float:
    """torch.cuda._sleep spins on the device clock; calibrate cycles per µs once."""
    if not _SLEEP_CAL:
        cyc = 2_000_000
        torch.cuda._sleep(cyc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda._sleep(cyc)
        e1.record()
        torch.cuda.synchronize()
        _SLEEP_CAL.append(cyc / (e0.elapsed_time(e1) * 1e3))
    return _SLEEP_CAL[0]


# The RRDB trunk runs as one persistent isr_conv_chain launch by default (ISR_CHAIN=0:
# one launch per conv); ISR_CHAIN_ACQUIRE=0 drops the per-tile agent-scope acquire and
# relies on the sc1 (L1-bypassing) activation loads alone (-1.5 % time).
import os as _os
CHAIN_DEFAULT = _os.environ.get("ISR_CHAIN", "1") == "1"
# The hand-off reads are sc1 LDS-DMA loads, which bypass L1; an agent-scope acquire only
# invalidates L1, so it adds nothing to them and costs ~1 ms per forward on the trunk kernel
# (per-wave fences).  Both modes are bitwise-tested (tests/test_gpu_chain.py).
CHAIN_ACQUIRE = _os.environ.get("ISR_CHAIN_ACQUIRE", "0") == "1"
# isr_conv_chain_variant: 0 = trunk.hip (production), 1 = the round-2 per-tile chain kernel, 2-5 the
# A/B forms documented at isr_conv_chain_variant in include/isr.h
CHAIN_VARIANT = int(_os.environ.get("ISR_CHAIN_VARIANT", "0"))


def _storage_exact(v: float, f16: int = 0) -> bool:
    """v is exactly representable in the activation storage type (bf16, or fp16 when f16)."""
    t = torch.tensor([v], dtype=torch.float32)
    return bool(t.to(torch.float16 if f16 else torch.bfloat16).to(torch.float32).item() == t.item())

# Batches of >= 2 (even) are split over this many HIP streams by default: two
# half-batch launch lists run concurrently, so one stream's kernel tail, prologue
# and HBM-bound epilogue overlap the other's MFMA main loop (+6 % on the
# 16 x 128² → 512² batch, tools/ab_split.py; outputs identical).
DEFAULT_STREAMS = 2


class GraphedPlan:
    """A plan's whole forward (every launch on every stream) captured once into a
    HIP graph for fixed input / output tensors and replayed per call: one graph
    launch instead of ~245 (x streams) ctypes launches, whose host cost (~15 us
    each) would otherwise bound a fast forward.  Outputs are identical to the
    eager plan (same kernels, same order per stream)."""

    def __init__(self, plan, x: torch.Tensor, out: torch.Tensor):
        self.plan, self.x, self.out = plan, x, out
        side = torch.cuda.Stream(x.device)
        side.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(side):  # warm-up outside capture (lazy attribute setup)
            plan.run(x, out)
        torch.cuda.current_stream(x.device).wait_stream(side)
        torch.cuda.synchronize(x.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            plan.run(x, out)

    def run(self) -> torch.Tensor:
        self.graph.replay()
        for c in self.plan.chains:  # outside the graph: a lagged, non-blocking give-up check
            c.poll()
        return self.out

    def verify(self) -> None:
        self.plan.verify()


def make_plan(gw: GeneratorWeights, n: int, h: int, w: int, device, x_u8: bool, out_u8: bool, mean, std,
              streams: int | None = None, chain: bool | None = None):
    """GeneratorPlan, or a SplitGeneratorPlan over `streams` (default DEFAULT_STREAMS, or 1
    with the chained trunk) HIP streams when the batch divides evenly."""
    chain = CHAIN_DEFAULT if chain is None else chain
    k = (1 if chain else DEFAULT_STREAMS) if streams is None else streams
    if k > 1 and n >= k and n % k == 0:
        return SplitGeneratorPlan(gw, n, h, w, device, x_u8, out_u8, mean, std, splits=k, chain=chain)
    return GeneratorPlan(gw, n, h, w, device, x_u8, out_u8, mean, std, chain=chain)


def get_plan(gw: GeneratorWeights, x: torch.Tensor, out_u8: bool, mean, std, streams: int | None = None,
             chain: bool | None = None):
    n, c, h, w = x.shape
    if c != 3:
        raise ValueError(f"generator expects 3 input channels, got {c}")
    key = (n, h, w, str(x.device), x.dtype == torch.uint8, out_u8, tuple(mean), tuple(std), streams, chain)
    plan = gw.buffers.get("plan")
    if plan is None or gw.buffers.get("plan_key") != key:
        gw.buffers["plan"] = None  # free the previous geometry first
        plan = make_plan(gw, n, h, w, x.device, x.dtype == torch.uint8, out_u8, mean, std, streams, chain)
        gw.buffers["plan"] = plan
        gw.buffers["plan_key"] = key
    return plan


def run_generator(gw: GeneratorWeights, x: torch.Tensor, *, out_u8: bool = False,
                  mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)) -> torch.Tensor:
    """x: NCHW [n,3,h,w] fp32 (normalised) or uint8 (Normalize fused) on the GPU."""
    x = x.contiguous()
    plan = get_plan(gw, x, out_u8, mean, std)
    out = torch.empty(plan.out_shape, dtype=plan.out_dtype, device=x.device)
    return plan.run(x, out)


def generator_flops(h: int, w: int, num_blocks: int = 16, n_scalers: int = 2) -> float:
    """Algorithmic FLOPs (2*MAC) of one generator forward on an h x w LR image."""
    px = h * w
    macs = px * 64 * 3 * 81  # conv0
    rdb = sum((64 + 32 * k) * 32 * 9 for k in range(4)) + 192 * 64 * 9
    macs += px * num_blocks * 3 * rdb
    macs += px * 64 * 64 * 9  # conv1
    p = px
    for _ in range(n_scalers):
        macs += p * 64 * 256 * 9
        p *= 4
    macs += p * 64 * 3 * 81  # conv2
    return 2.0 * macs
