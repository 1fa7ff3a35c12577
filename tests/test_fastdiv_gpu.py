"""The render kernel's fast correctly-rounded reciprocal / quotient (csrc/rtx_fastdiv.h)
against the hardware's IEEE `1/x` and `a/b`: every one of the 2^32 reciprocal inputs in the
fast domain and 2^33 random + near-halfway quotients (tools/validate_fastdiv.hip)."""
import json
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def test_fast_division_is_ieee_exact(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = tmp_path / "validate_fastdiv"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fno-fast-math",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", f"-I{ROOT / 'gp1_raytracer_2223_amd' / 'csrc'}",
                    str(ROOT / "tools" / "validate_fastdiv.hip"), "-o", str(exe)], check=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    rows = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(rows) == 9, out.stdout + out.stderr
    assert all(r["mismatches"] == 0 and r["tested"] > 0 for r in rows), rows
    assert out.returncode == 0
