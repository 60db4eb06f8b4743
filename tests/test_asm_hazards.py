"""The GEMM k-loops read LDS through asm statements (csrc/common.h
lds_read_*_async) and retire the reads themselves; hipcc must not touch the
destination registers in between (a spill store there read a fragment
before it landed).  tools/lgkm_check.py finds such reads in the gfx950
assembly: checked here on a synthetic listing and on gemm.hip as built."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from lgkm_check import check  # noqa: E402

SYNTH = """
_Zgood:
	ds_read_b64_tr_b16 v[10:11], v2
	ds_read_b64_tr_b16 v[12:13], v3
	s_waitcnt lgkmcnt(1)
	v_mov_b32_e32 v20, v10
	s_waitcnt lgkmcnt(0)
	v_mfma_f32_16x16x32_bf16 v[0:3], v[10:13], v[10:13], v[0:3]
_Zbad:
	ds_read_b128 v[40:43], v2
	scratch_store_dwordx4 off, v[40:43], off
	s_waitcnt lgkmcnt(0)
_Zoverwritten:
	ds_read_b32 v7, v2
	v_mov_b32_e32 v7, 0
	v_add_u32_e32 v8, v7, v7
_Zloopcarried:
.LBB0_1:
	v_mov_b32_e32 v30, v20
	s_waitcnt lgkmcnt(0)
	ds_read_b64 v[20:21], v2
	s_cbranch_scc1 .LBB0_1
	s_waitcnt lgkmcnt(0)
_Zsmem:
	ds_read_b64 v[50:51], v2
	s_load_dwordx2 s[4:5], s[0:1], 0x0
	s_waitcnt lgkmcnt(1)
	v_mov_b32_e32 v52, v50
	s_waitcnt lgkmcnt(0)
"""


def test_checker_on_synthetic_listing(tmp_path):
    p = tmp_path / "s.s"
    p.write_text(SYNTH)
    bad = check(str(p))
    # _Zloopcarried: v20 is read at the loop head while the previous
    # iteration's ds_read of it is still in flight (found via the back-edge);
    # _Zsmem: lgkmcnt(1) with a scalar load pending retires no LDS read
    assert set(bad) == {"_Zbad", "_Zloopcarried", "_Zsmem"}
    assert "scratch_store" in bad["_Zbad"][0][1]


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_gemm_kernels_have_no_early_reads(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    src = os.path.join(ROOT, "smer_music_generation_amd", "csrc", "gemm.hip")
    out = tmp_path / "gemm.s"
    from smer_music_generation_amd.csrc.build import NO_PACKED_F32
    r = subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "include"), src, "-o", str(out)] + NO_PACKED_F32,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    bad = {f: v for f, v in check(str(out)).items() if "gemm" in f}
    assert not bad, bad


def test_library_has_no_packed_f32_instructions():
    """DESIGN.md section 8 (round 6): packed-FP32 VALU results (v_pk_fma_f32 /
    v_pk_mul_f32 / v_pk_add_f32) came out wrong in lanes 48-63 while another
    workgroup on the same CU streamed LDS-DMA, which made the overlapped
    train step non-repeatable.  The library is built without them
    (csrc/build.py NO_PACKED_F32); this scans the shipped gfx950 code."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pk_scan
    lib = os.path.join(ROOT, "smer_music_generation_amd", "libsmer_hip.so")
    if not os.path.exists(lib) or not pk_scan.tools_available():
        pytest.skip("built library or LLVM tools absent")
    n, found = pk_scan.scan(lib)
    assert n >= 5, "expected the gfx950 code objects of every .hip source, found %d" % n
    assert not found, "packed-FP32 instructions in %s" % sorted(found.items(), key=lambda x: -x[1])[:5]
