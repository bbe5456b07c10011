"""tools/check_lds_waits.py — the build-time check of hand-counted LDS waits — on
small gfx950 assembly snippets: it must pass correctly waited reads, catch a read of a fragment
before its wait (also across a loop back-edge), an SMEM load under a counted wait, a non-LDS write
into a register an LDS read still targets, and a kernel with scratch.  CPU only: the production
kernels themselves are checked by image_super_resolution_amd/_build.py on every full build."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import check_lds_waits as C  # noqa: E402


def _kernel(body: str, scratch: int = 0) -> str:
    return (f"_Z1kv: ; @_Z1kv\n{body}\n\ts_endpgm\n.Lfunc_end0:\n"
            f"\t.amdhsa_kernel _Z1kv\n\t\t.amdhsa_private_segment_fixed_size {scratch}\n\t.end_amdhsa_kernel\n")


ASM_READ = "\t;;#ASMSTART\n\tds_read_b64_tr_b16 v[4:5], v2 offset:0\n\t;;#ASMEND\n"


def test_counted_wait_passes():
    body = ASM_READ + "\tds_read_b64_tr_b16 v[6:7], v2 offset:128\n\ts_waitcnt lgkmcnt(1)\n" \
        "\tv_mfma_f32_32x32x16_bf16 a[0:15], v[4:7], v[8:11], a[0:15]\n"
    # v[6:7] is the younger read, still allowed in flight by lgkmcnt(1): the MFMA reads it -> error
    assert C.check_asm(_kernel(body), "t")
    body_ok = ASM_READ + "\tds_read_b64_tr_b16 v[6:7], v2 offset:128\n\ts_waitcnt lgkmcnt(1)\n" \
        "\tv_add_f32_e32 v20, v4, v5\n\ts_waitcnt lgkmcnt(0)\n\tv_add_f32_e32 v21, v6, v7\n"
    assert C.check_asm(_kernel(body_ok), "t") == []


def test_read_before_wait_is_caught():
    errs = C.check_asm(_kernel(ASM_READ + "\tv_add_f32_e32 v20, v4, v5\n"), "t")
    assert errs and "before the LDS read" in errs[0]


def test_smem_under_counted_wait_is_caught():
    body = ASM_READ + "\ts_load_dword s4, s[0:1], 0x0\n\ts_waitcnt lgkmcnt(1)\n\tv_mov_b32_e32 v9, s4\n"
    errs = C.check_asm(_kernel(body), "t")
    assert any("SMEM" in e for e in errs)


def test_overwrite_of_pending_destination_is_caught():
    errs = C.check_asm(_kernel(ASM_READ + "\tv_mov_b32_e32 v5, 0\n\ts_waitcnt lgkmcnt(0)\n"), "t")
    assert errs and "still in flight" in errs[0]
    # a second LDS read into the same register is fine (one wave's LDS reads return in order)
    ok = ASM_READ + "\tds_read_b64_tr_b16 v[4:5], v3 offset:0\n\ts_waitcnt lgkmcnt(0)\n\tv_add_f32_e32 v9, v4, v5\n"
    assert C.check_asm(_kernel(ok), "t") == []


def test_read_ahead_across_back_edge():
    """A read issued at the bottom of an iteration and consumed at the top of the next one before
    any wait: only a CFG walk that follows the back-edge sees it."""
    bad = ("\ts_mov_b32 s6, 4\n.LBB0_1:\n\tv_add_f32_e32 v20, v4, v5\n" + ASM_READ +
           "\ts_sub_i32 s6, s6, 1\n\ts_cmp_lg_u32 s6, 0\n\ts_cbranch_scc1 .LBB0_1\n\ts_waitcnt lgkmcnt(0)\n")
    errs = C.check_asm(_kernel(bad), "t")
    assert errs and "v_add_f32_e32 v20, v4, v5" in errs[0]
    good = bad.replace(".LBB0_1:\n", ".LBB0_1:\n\ts_waitcnt lgkmcnt(0)\n")
    assert C.check_asm(_kernel(good), "t") == []


def test_scratch_is_an_error():
    errs = C.check_asm(_kernel("\tv_mov_b32_e32 v1, 0\n", scratch=8), "t")
    assert errs and "scratch" in errs[0]
