"""The packed owner-segment records (fluere_amd/csrc/seg.h) round-trip every
field of a spilled packet (kern.h `Spill`, written by k_parse_spill /
k_parse_agg / k_slow, read by k_merge_spill / k_merge_partials): a host build
of tests/native/seg_roundtrip.cpp.  The GPU parity tests cover the kernels
that use them (test_full_size_parity, the spill/overflow tests)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_seg_pack_round_trip(tmp_path):
    exe = tmp_path / "seg_roundtrip"
    src = os.path.join(HERE, "native", "seg_roundtrip.cpp")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-o", str(exe), src], check=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout
