"""Inline-asm / MFMA hazard scan of the built kernels (CPU only, no GPU).

The compiler's hazard recognizer does not see inside inline asm: an asm VALU that writes a register an
in-flight MFMA still reads as its accumulator input, or reads an MFMA result too early, gets no wait
states.  Such a build renders wrong frames that differ run to run (63962d3) and shows no other
symptom.  The library build keeps each object's gfx950 assembly (csrc/Makefile: build/<src>.gfx950.s,
the same compile as the object); tools/asm_hazards.py must report no candidate in any of them, and must
report the one planted in tests/asm_hazard_plant.hip.
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sg-nerf_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(ROOT, "tools"))
import asm_hazards  # noqa: E402

needs_hipcc = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


@needs_hipcc
def test_scan_flags_a_planted_hazard(tmp_path):
    out = tmp_path / "plant.s"
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-S",
                           os.path.join(ROOT, "tests", "asm_hazard_plant.hip"), "-o", str(out)])
    found = asm_hazards.scan(out.read_text())
    assert found, "the planted asm read of an MFMA result was not reported"


def test_scan_ignores_compiler_visible_reads():
    """The same instruction sequence without the inline-asm markers is the compiler's own (it padded it)."""
    text = "\n".join(["v_mfma_f32_16x16x32_f16 v[0:3], v[4:7], v[8:11], v[0:3]",
                      "s_nop 7", "v_add_f32_e32 v12, v0, v0"])
    assert asm_hazards.scan(text) == []
    planted = text.replace("v_add_f32_e32", ";;#ASMSTART\nv_add_f32_e32") + "\n;;#ASMEND"
    assert len(asm_hazards.scan(planted)) == 1


@needs_hipcc
def test_built_kernels_have_no_hazard_candidates():
    # up to date after build(): a no-op; otherwise (re)builds the objects and their listings
    subprocess.check_call(["make", "-s", "-C", CSRC, "-j", str(min(8, os.cpu_count() or 1))])
    listings = sorted(glob.glob(os.path.join(CSRC, "build", "*.gfx950.s")))
    assert len(listings) >= 10, listings
    scanned_asm = 0
    for p in listings:
        text = open(p).read()
        if "v_mfma" not in text:
            continue
        scanned_asm += text.count(";;#ASMSTART")
        found = asm_hazards.scan(text)
        assert not found, f"{os.path.basename(p)}: {len(found)} inline-asm/MFMA hazard candidates, e.g. {found[:3]}"
    assert scanned_asm > 100, "no inline asm beside MFMAs was scanned (listings without asm markers?)"
