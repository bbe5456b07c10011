"""Video super-resolution path (BASELINE configs[4]).

Mirrors the reference's video branch — rs.py:54-76 (decode → Normalize → model
→ TanhToArrayImage → RGB2BGR → FFMPEG_recorder), utils/datasets.py:431-463
(`dataset_for_inference`: frames as uint8 CHW, fps from the container) and
utils/ffmpeg.py:28-140 (`FFMPEG_recorder`: raw bgr24 frames piped to an ffmpeg
encoder, bitrate ∝ output megapixels) — rebuilt around the MI355X path:

* the per-batch forward (uint8 HWC RGB in → Normalize fused into the head
  kernel → RRDB trunk → tail + TanhToArrayImage fused → BGR HWC uint8 out) is
  one `GeneratorPlan` whose ~245 kernel launches, plus the layout copies on
  either side, are captured once into a HIP graph and replayed per batch
  (torch.cuda.CUDAGraph over the HIP stream: no per-frame CPU launch cost);
* frames are staged through pinned host buffers, two output slots deep, so the
  device→host copy of batch i and the encoder write of batch i-1 overlap the
  forward of batch i+1; encoding runs on a writer thread;
* decode / encode use the ffmpeg binary through raw pipes when it is installed
  (as the reference does); `RawVideoReader` / `RawRecorder` read and write
  headerless rgb24 / bgr24 files and `SyntheticVideo` generates frames, so the
  pipeline is testable and benchmarkable on a machine without ffmpeg.

Reference bugs deliberately not reproduced: the frame is
normalised once (rs.py:63 normalises before a TorchScript Model that normalises
again) and quantised to uint8 once (rs.py:65 re-applies TanhToArrayImage to
the model's uint8 output); frames are read in order (the reference's
DataLoader uses shuffle=True but `__getitem__` ignores the index).
"""
from __future__ import annotations

import math
import platform
import queue
import shutil
import subprocess
import threading
from pathlib import Path
from typing import Iterator

import numpy as np
import torch

from . import engine

VID_FORMATS = ('.mp4', '.avi', '.mkv', '.mov', '.wmv', '.flv', '.webm', '.mpeg', '.mpg', '.m4v', '.ts')


def have_ffmpeg() -> bool:
    return shutil.which("ffmpeg") is not None and shutil.which("ffprobe") is not None


# ----------------------------------------------------------------------------- sources
class FFmpegVideoReader:
    """Decoded uint8 HWC RGB frames of a video file via an ffmpeg rawvideo pipe
    (the role of torchvision's VideoReader in utils/datasets.py:431-453)."""

    def __init__(self, src: str | Path):
        if not have_ffmpeg():
            raise RuntimeError("FFmpegVideoReader needs the ffmpeg and ffprobe binaries")
        src = Path(src)
        probe = subprocess.run(["ffprobe", "-v", "error", "-select_streams", "v:0", "-show_entries",
                                "stream=width,height,r_frame_rate,nb_frames,duration", "-of",
                                "default=noprint_wrappers=1", src.as_posix()],
                               capture_output=True, text=True, check=True).stdout
        meta = dict(line.split("=", 1) for line in probe.strip().splitlines() if "=" in line)
        self.width, self.height = int(meta["width"]), int(meta["height"])
        num, den = (meta.get("r_frame_rate", "30/1").split("/") + ["1"])[:2]
        self.fps = float(num) / float(den or 1)
        nb = meta.get("nb_frames", "N/A")
        dur = meta.get("duration", "N/A")
        self.total_frame = int(nb) if nb.isdigit() else (int(self.fps * float(dur)) if dur != "N/A" else 0)
        self.src = src

    def __len__(self):
        return self.total_frame

    def __iter__(self) -> Iterator[np.ndarray]:
        cmd = ["ffmpeg", "-v", "quiet", "-i", self.src.as_posix(), "-f", "rawvideo", "-pix_fmt", "rgb24", "pipe:"]
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE)
        n = self.width * self.height * 3
        try:
            while True:
                buf = proc.stdout.read(n)
                if len(buf) < n:
                    break
                yield np.frombuffer(buf, np.uint8).reshape(self.height, self.width, 3)
        finally:
            proc.stdout.close()
            proc.wait()


class RawVideoReader:
    """Headerless rgb24 frames (H x W x 3 uint8, back to back) from a file."""

    def __init__(self, src: str | Path, width: int, height: int, fps: float = 30.0):
        self.src, self.width, self.height, self.fps = Path(src), width, height, fps
        size = self.src.stat().st_size
        fb = width * height * 3
        if size % fb:
            raise ValueError(f"{src}: {size} bytes is not a whole number of {width}x{height} rgb24 frames")
        self.total_frame = size // fb

    def __len__(self):
        return self.total_frame

    def __iter__(self) -> Iterator[np.ndarray]:
        mm = np.memmap(self.src, np.uint8, "r", shape=(self.total_frame, self.height, self.width, 3))
        for i in range(self.total_frame):
            yield np.asarray(mm[i])


class SyntheticVideo:
    """`frames` smooth moving uint8 RGB frames (benchmarks / tests; no decoder)."""

    def __init__(self, width: int, height: int, frames: int, fps: float = 30.0, seed: int = 0):
        self.width, self.height, self.total_frame, self.fps = width, height, frames, fps
        g = np.random.default_rng(seed)
        yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
        self._base = [(np.sin(xx / (17 + 9 * c) + c) * np.cos(yy / (13 + 7 * c)) + 1) * 100 for c in range(3)]
        self._noise = g.integers(0, 40, size=(height, width, 3), dtype=np.uint8)

    def __len__(self):
        return self.total_frame

    def __iter__(self) -> Iterator[np.ndarray]:
        for i in range(self.total_frame):
            s = i % 32
            f = np.stack([np.roll(b, s, axis=1) for b in self._base], axis=-1).astype(np.uint8)
            yield f + self._noise


def open_video(src: str | Path, width: int | None = None, height: int | None = None, fps: float = 30.0):
    """`dataset_for_inference` equivalent: ffmpeg for container formats, raw for .rgb/.raw."""
    src = Path(src)
    if src.suffix.lower() in (".rgb", ".raw", ".rgb24"):
        if not (width and height):
            raise ValueError("raw rgb24 input needs --video_size WxH")
        return RawVideoReader(src, width, height, fps)
    return FFmpegVideoReader(src)


# ----------------------------------------------------------------------------- sinks
def _gpu_vendor() -> str:
    try:
        return "AMD" if torch.version.hip else ("NVIDIA" if torch.cuda.is_available() else "")
    except Exception:  # noqa: BLE001
        return ""


def _bitrate_mbps(dims, fps) -> float:
    """Target bitrate in Mbit/s (utils/ffmpeg.py:59-61): 20 Mbit/s for a 4K frame at 30 fps, scaled
    by the frame area and by the frame-rate ratio, which is never taken below 1."""
    rate_factor = round(fps / 30, 3)
    if rate_factor < 1:
        rate_factor = 1
    return round(20 * (math.prod(dims) / (3840 * 2160)) * rate_factor, 3)


def _srt_entry(index: int, t0: str, t1: str, text: str) -> str:
    return f"{index}\n{t0} --> {t1}\n{text}\n\n"


class FFMPEG_recorder:  # noqa: N801  (reference class name, utils/ffmpeg.py:28)
    """utils/ffmpeg.py:28-140: raw bgr24 frames piped into an ffmpeg encoder process.

    The public surface is the reference's (constructor arguments, `bitRate`, `cmd`,
    `subtitleContent`, writeFrame / writeSubtitle / addSubtitle / addAudio / stopRecorder) and so is
    what ffmpeg receives (tests/test_video_cpu.py pins the argv, bitrate and timecodes).  The encoder
    is hevc_vaapi on a Linux host with an AMD GPU when ffmpeg offers it (the reference's preference
    for that platform), else libx264."""

    def __init__(self, save_path=None, videoDimensions=(1280, 720), fps=30, codec: str | None = None,
                 dry_run: bool = False):
        self.save_path = save_path
        self.dimension = videoDimensions
        self.fps = fps
        if codec is None:
            amd_linux = platform.uname().system == "Linux" and _gpu_vendor() == "AMD"
            codec = "hevc_vaapi" if amd_linux and _has_encoder("hevc_vaapi") else "libx264"
        self.codec = codec
        out_path = save_path.replace(" ", "_") if save_path else save_path  # ffmpeg target without spaces
        self.countFrame = 0
        self.startTime = 0.
        self.bitRate = _bitrate_mbps(self.dimension, self.fps)
        self.subtitleContent = ''
        width, height = self.dimension
        source = ['-s', f'{width}x{height}', '-pixel_format', 'bgr24', '-f', 'rawvideo', '-r', f'{self.fps}',
                  '-i', 'pipe:']
        sink = ['-vcodec', f'{self.codec}', '-pix_fmt', 'yuv420p', '-b:v', f'{self.bitRate}M', f'{out_path}']
        self.cmd = ['ffmpeg', '-v', 'quiet', '-y', *source, *sink]
        self.process = None
        if dry_run:
            return
        if shutil.which("ffmpeg") is None:
            raise RuntimeError("FFMPEG_recorder needs the ffmpeg binary (use RawRecorder without it)")
        self.process = subprocess.Popen(self.cmd, stdin=subprocess.PIPE)

    def writeFrame(self, image=None):  # noqa: N802
        """image: ndarray uint8 HWC BGR."""
        self.process.stdin.write(np.ascontiguousarray(image).tobytes())

    @staticmethod
    def second_to_timecode(x=0.) -> str:
        """SubRip timecode HH:MM:SS,mmm of x seconds, milliseconds truncated (utils/ffmpeg.py:81-89;
        float divmod is exact, so x mod 1 equals the reference's chained remainders)."""
        whole, frac = divmod(x, 1)
        hours, rest = divmod(int(whole), 3600)
        minutes, seconds = divmod(rest, 60)
        return f"{hours:02d}:{minutes:02d}:{seconds:02d},{int(frac * 1000.):03d}"

    def writeSubtitle(self, title='', fps=30):  # noqa: N802
        """One SubRip cue of 1/fps seconds at the running clock (utils/ffmpeg.py:91-100)."""
        t0 = self.startTime
        self.startTime = t0 + 1 / fps
        self.subtitleContent += _srt_entry(self.countFrame, self.second_to_timecode(t0),
                                           self.second_to_timecode(self.startTime), title or "UTC2")
        self.countFrame += 1

    def addSubtitle(self, hardSubtitle=False):  # noqa: N802,N803
        """Mux (or burn in, hardSubtitle) the collected cues into '<name>with_sub.mp4'."""
        muxed = self.save_path.replace('.mp4', 'with_sub.mp4')
        srt = muxed.replace('.mp4', '.srt')
        Path(srt).write_text(self.subtitleContent)
        head = ["ffmpeg", "-hide_banner", "-i", self.save_path]
        if hardSubtitle:
            tail = ["-c:v", "copy", "-vf", f"subtitles={srt}"]
        else:
            tail = ["-i", srt, "-c:v", "copy", "-c:s", "mov_text", "-metadata:s:s:0", "language=eng"]
        return subprocess.run([*head, *tail, muxed])

    def addAudio(self, audio_src):  # noqa: N802
        """Copy the video stream and take the audio of `audio_src` into '<name>_audio.mp4'; 0 when
        there is no such file, else 1."""
        src = Path(audio_src)
        if not src.is_file():
            return 0
        target = self.save_path.replace(".mp4", "_audio.mp4")
        streams = ["-c:v", "copy", "-map", "0:v", "-map", "1:a"]
        subprocess.run(["ffmpeg", "-i", self.save_path, "-i", src.as_posix(), *streams, "-y", target])
        return 1

    def stopRecorder(self):  # noqa: N802
        if self.process is None:
            return
        self.process.stdin.close()
        self.process.wait()


def _has_encoder(name: str) -> bool:
    if shutil.which("ffmpeg") is None:
        return False
    try:
        out = subprocess.run(["ffmpeg", "-hide_banner", "-encoders"], capture_output=True, text=True, timeout=10).stdout
    except Exception:  # noqa: BLE001
        return False
    return f" {name} " in out


class RawRecorder:
    """Writes headerless bgr24 frames to a file (FFMPEG_recorder's pipe payload)."""

    def __init__(self, save_path, videoDimensions=(1280, 720), fps=30):  # noqa: N803
        self.save_path, self.dimension, self.fps = str(save_path), videoDimensions, fps
        self._f = open(self.save_path, "wb")
        self.frames = 0

    def writeFrame(self, image):  # noqa: N802
        self._f.write(np.ascontiguousarray(image).tobytes())
        self.frames += 1

    def stopRecorder(self):  # noqa: N802
        self._f.close()

    def addAudio(self, audio_src):  # noqa: N802
        return 0


class NullRecorder:
    """Counts frames (benchmarks: measures the pipeline without an encoder)."""

    def __init__(self, *a, **k):
        self.frames = 0

    def writeFrame(self, image):  # noqa: N802
        self.frames += 1

    def stopRecorder(self):  # noqa: N802
        pass

    def addAudio(self, audio_src):  # noqa: N802
        return 0


# ----------------------------------------------------------------------------- the GPU pipeline
class FrameUpscaler:
    """uint8 HWC RGB frame batches → uint8 HWC BGR super-resolved frames on the
    HIP generator, one captured HIP graph per batch geometry.

    `gw` is an engine.GeneratorWeights (tiler.runner_for(model).gw); `mean` /
    `std` the Normalize constants fused into the head kernel."""

    def __init__(self, gw: engine.GeneratorWeights, height: int, width: int, batch: int = 1, mean=(0.485, 0.456, 0.406),
                 std=(0.229, 0.224, 0.225), device="cuda", graph: bool = True):
        self.device = torch.device(device)
        self.batch, self.h, self.w = batch, height, width
        self.scale = 2 ** len(gw.scalers)
        self.plan = engine.make_plan(gw, batch, height, width, self.device, True, True, mean, std)
        H, W = height * self.scale, width * self.scale
        self.out_hw = (H, W)
        self.x_hwc = torch.zeros((batch, height, width, 3), dtype=torch.uint8, device=self.device)
        self.x = torch.empty((batch, 3, height, width), dtype=torch.uint8, device=self.device)
        self.y = torch.empty(self.plan.out_shape, dtype=torch.uint8, device=self.device)
        self.bgr = torch.empty((batch, H, W, 3), dtype=torch.uint8, device=self.device)
        self.stream = torch.cuda.Stream(self.device)
        self.graph = None
        with torch.cuda.stream(self.stream):
            for _ in range(2):  # warm-up: lazily set kernel attributes, allocator pools
                self._body()
        self.stream.synchronize()
        if graph:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=self.stream):
                self._body()
            self.stream.synchronize()

    def _body(self):
        self.x.copy_(self.x_hwc.permute(0, 3, 1, 2))
        self.plan.run(self.x, self.y)
        self.bgr.copy_(self.y.flip(1).permute(0, 2, 3, 1))  # RGB2BGR + CHW→HWC (utils/datasets.py RGB2BGR)

    def run_async(self):
        """Forward of whatever x_hwc holds, on self.stream."""
        with torch.cuda.stream(self.stream):  # replay() launches on the current stream
            if self.graph is not None:
                self.graph.replay()
            else:
                self._body()

    def __call__(self, frames_hwc: torch.Tensor) -> torch.Tensor:
        """Synchronous convenience: uint8 [b,h,w,3] RGB (host or device) → device [b,H,W,3] BGR."""
        b = frames_hwc.shape[0]
        if b > self.batch or tuple(frames_hwc.shape[1:]) != (self.h, self.w, 3):
            raise ValueError(f"frames {tuple(frames_hwc.shape)} do not fit the plan {(self.batch, self.h, self.w, 3)}")
        with torch.cuda.stream(self.stream):
            self.x_hwc[:b].copy_(frames_hwc, non_blocking=True)
            if b < self.batch:
                self.x_hwc[b:].zero_()
        self.run_async()
        self.stream.synchronize()
        with torch.cuda.stream(self.stream):
            self.plan.verify()  # a persistent-chain give-up raises before the frames are handed out
        return self.bgr[:b]


class VideoUpscaler:
    """rs.py:54-76 as a streaming pipeline: source frames → FrameUpscaler →
    recorder.  Two pinned input and two pinned output slots: while the GPU runs
    batch i, the host decodes batch i+1 into the other input slot and the writer
    thread encodes batch i-1 from the other output slot."""

    def __init__(self, up: FrameUpscaler):
        self.up = up
        b, h, w = up.batch, up.h, up.w
        H, W = up.out_hw
        self.pin_in = [torch.empty((b, h, w, 3), dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.pin_out = [torch.empty((b, H, W, 3), dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.h2d_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.d2h_done = [torch.cuda.Event(), torch.cuda.Event()]
        # per output slot: the chains' give-up counts, copied right after that batch's forward
        # (outside the captured graph) and checked by the writer before the batch is encoded
        self.chains = list(up.plan.chains)
        self.pin_state = [torch.zeros(max(1, len(self.chains)), dtype=torch.int32).pin_memory() for _ in range(2)]

    def run(self, frames, recorder, max_frames: int | None = None) -> int:
        """Upscale every frame of `frames` (iterable of uint8 HWC RGB arrays) into
        `recorder.writeFrame` (BGR HWC).  Returns the number of frames written."""
        up, b = self.up, self.up.batch
        q: queue.Queue = queue.Queue()
        out_free = [threading.Event(), threading.Event()]
        for e in out_free:
            e.set()
        err: list[BaseException] = []

        def writer():
            while True:
                item = q.get()
                if item is None:
                    return
                slot, n = item
                try:
                    if not err:
                        self.d2h_done[slot].synchronize()
                        for k, c in enumerate(self.chains):  # raises engine.ChainFailed
                            c.check_count(int(self.pin_state[slot][k]))
                        arr = self.pin_out[slot].numpy()
                        for i in range(n):
                            recorder.writeFrame(arr[i])
                except BaseException as e:  # noqa: BLE001
                    err.append(e)
                finally:
                    out_free[slot].set()

        th = threading.Thread(target=writer, daemon=True)
        th.start()
        written, slot = 0, 0
        it = iter(frames)
        try:
            while not err:
                self.h2d_done[slot].synchronize()  # the H2D copy of batch i-2 has left this input slot
                pin_np = self.pin_in[slot].numpy()
                n = 0
                while n < b and (max_frames is None or written + n < max_frames):
                    try:
                        pin_np[n] = next(it)
                    except StopIteration:
                        break
                    n += 1
                if n == 0:
                    break
                if n < b:
                    pin_np[n:] = 0
                out_free[slot].wait()  # the writer is done with batch i-2's output slot
                out_free[slot].clear()
                with torch.cuda.stream(up.stream):
                    up.x_hwc.copy_(self.pin_in[slot], non_blocking=True)
                    self.h2d_done[slot].record(up.stream)
                up.run_async()
                with torch.cuda.stream(up.stream):
                    for k, c in enumerate(self.chains):
                        c.snapshot(self.pin_state[slot][k:k + 1])
                    self.pin_out[slot].copy_(up.bgr, non_blocking=True)
                    self.d2h_done[slot].record(up.stream)
                q.put((slot, n))
                written += n
                slot ^= 1
        finally:
            q.put(None)
            th.join()
        if err:
            raise err[0]
        return written
