"""Host-side video plumbing (video.py): FFMPEG_recorder mirror (utils/ffmpeg.py:28-140),
raw rgb24 reader / bgr24 recorder, synthetic source.  No GPU, no ffmpeg needed."""
import numpy as np
import pytest

from image_super_resolution_amd import video


@pytest.mark.parametrize("dims,fps,rate", [((3840, 2160), 30, 20.0), ((7680, 4320), 60, 160.0),
                                           ((1920, 1080), 24, 5.0), ((1280, 720), 45, 3.333)])
def test_recorder_bitrate_and_command(dims, fps, rate):
    # utils/ffmpeg.py:59-61: 20 Mb/s per 4K frame area, scaled by fps/30 when fps >= 30
    r = video.FFMPEG_recorder("out dir/x.mp4", dims, fps, codec="libx264", dry_run=True)
    assert r.bitRate == pytest.approx(rate, abs=1e-3)
    assert r.cmd[:4] == ["ffmpeg", "-v", "quiet", "-y"]
    assert r.cmd[r.cmd.index("-s") + 1] == f"{dims[0]}x{dims[1]}"
    assert r.cmd[r.cmd.index("-pixel_format") + 1] == "bgr24"
    assert r.cmd[r.cmd.index("-b:v") + 1] == f"{r.bitRate}M"
    assert r.cmd[-1] == "out_dir/x.mp4"  # spaces replaced (utils/ffmpeg.py:55-56)


def test_timecode_and_subtitles():
    assert video.FFMPEG_recorder.second_to_timecode(3725.25) == "01:02:05,250"
    r = video.FFMPEG_recorder("a.mp4", (64, 32), 30, codec="libx264", dry_run=True)
    r.writeSubtitle("hi", fps=10)
    r.writeSubtitle(fps=10)
    assert r.subtitleContent == "0\n00:00:00,000 --> 00:00:00,100\nhi\n\n1\n00:00:00,100 --> 00:00:00,200\nUTC2\n\n"


def test_raw_roundtrip(tmp_path):
    frames = [np.random.default_rng(i).integers(0, 256, (6, 10, 3), dtype=np.uint8) for i in range(3)]
    src = tmp_path / "in.rgb"
    src.write_bytes(b"".join(f.tobytes() for f in frames))
    rd = video.open_video(src, 10, 6, 25.0)
    assert len(rd) == 3 and rd.fps == 25.0
    got = list(rd)
    assert all(np.array_equal(a, b) for a, b in zip(got, frames))
    rec = video.RawRecorder(tmp_path / "out.bgr", (10, 6), 25)
    for f in got:
        rec.writeFrame(f[..., ::-1])
    rec.stopRecorder()
    back = np.frombuffer((tmp_path / "out.bgr").read_bytes(), np.uint8).reshape(3, 6, 10, 3)
    assert np.array_equal(back[..., ::-1], np.stack(frames))
    with pytest.raises(ValueError):
        video.open_video(src)  # raw input needs its size
    (tmp_path / "bad.rgb").write_bytes(b"\0" * 7)
    with pytest.raises(ValueError):
        video.RawVideoReader(tmp_path / "bad.rgb", 10, 6)


def test_synthetic_video():
    sv = video.SyntheticVideo(40, 24, 5)
    fr = list(sv)
    assert len(fr) == 5 and fr[0].shape == (24, 40, 3) and fr[0].dtype == np.uint8
    assert not np.array_equal(fr[0], fr[1])
