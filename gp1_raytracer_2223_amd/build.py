"""In-tree native build (no cmake/ninja, no JIT cache): explicit g++/gcc/hipcc lines.

Outputs (git-ignored, travel to the GPU box with the gpurun snapshot):
  gp1_raytracer_2223_amd/lib/librtx_host.so   C++ host scene layer (g++)
  gp1_raytracer_2223_amd/lib/librtx_hip.so    HIP render path for gfx950 (hipcc)
  oracle/_build/librtx_oracle.so              C restatement (test infrastructure)
  oracle/_ref/ref_harness                     the reference's own sources (test infra,
                                              only when /root/reference exists)

Every float-producing compile uses -ffp-contract=off and no fast-math: the reference is
MSVC /fp:precise x64 (no FMA contraction) and parity is bit-level.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
LIB = PKG / "lib"
CSRC = PKG / "csrc"
INC = REPO / "include"
ORACLE = REPO / "oracle"
REFERENCE = Path("/root/reference")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RTX_OFFLOAD_ARCH", "gfx950")


def _run(cmd: list[str], cwd: Path | None = None) -> None:
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True, cwd=cwd)


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def build_host(force: bool = False) -> Path:
    LIB.mkdir(exist_ok=True)
    out = LIB / "librtx_host.so"
    srcs = [CSRC / "host" / "scene.cpp", CSRC / "host" / "host_api.cpp", CSRC / "host" / "view.cpp"]
    deps = srcs + list((CSRC / "host").glob("*.h")) + [INC / "rtx.h", INC / "rtx_host.h", INC / "rtx_view.h",
                                                         Path(__file__)]
    if force or _stale(out, deps):
        _run(["g++", "-std=c++17", "-O3", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-pthread",
              "-Wall", "-Wextra", f"-I{INC}", *srcs, "-o", out, "-ldl"])
    return out


def build_hip(force: bool = False) -> Path:
    LIB.mkdir(exist_ok=True)
    out = LIB / "librtx_hip.so"
    srcs = [CSRC / "rtx_hip.hip", CSRC / "rtx_policy.hip", CSRC / "rtx_anim.hip", CSRC / "rtx_anim_host.hip",
            CSRC / "rtx_group.cpp"]
    deps = srcs + list(CSRC.glob("*.h")) + [INC / "rtx.h", INC / "rtx_diag.h", Path(__file__)]   # flags live here
    if force or _stale(out, deps):
        # -fno-slp-vectorize: the SLP packer turns independent f32 ops into v_pk_* plus
        # v_mov shuffles; measured 8 % slower on the render kernel (profiles/r01/ablate_*.txt).
        # -structurizecfg-skip-uniform-regions: wave-uniform loops and branches (every loop of
        # the BVH walk) stay plain s_cbranch_scc instead of being structurized into SGPR
        # lane-mask phis (s_cselect -1/0 + s_and vcc, exec per exit): -6 % SALU per wave.
        _run([HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-O3", "-ffp-contract=off",
              "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize",
              "-mllvm", "-structurizecfg-skip-uniform-regions=true",
              "-DRTX_MIN_WAVES_PER_EU=6", "-fPIC", "-shared", "-pthread",
              "-Wall", f"-I{INC}", f"-I{CSRC}", *srcs, "-o", out])
    return out


def build_cli(force: bool = False) -> Path:
    """Headless C++ host program over both libraries (lib/rtx_render)."""
    out = LIB / "rtx_render"
    src = CSRC / "cli" / "rtx_render.cpp"
    deps = [src, CSRC / "cli" / "benchmark.h", INC / "rtx_renderer.hpp", INC / "rtx.h", INC / "rtx_host.h", LIB / "librtx_hip.so",
            LIB / "librtx_host.so"]
    if force or _stale(out, deps):
        _run(["g++", "-std=c++17", "-O2", "-Wall", f"-I{INC}", src, "-o", out, f"-L{LIB}", "-lrtx_hip", "-lrtx_host",
              "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"])
    return out


def build_view(force: bool = False) -> Path:
    """The SDL viewer (lib/rtx_view): SDL2 is dlopen'ed at run time, nothing links against it."""
    out = LIB / "rtx_view"
    src = CSRC / "cli" / "rtx_view.cpp"
    deps = [src, CSRC / "cli" / "benchmark.h", INC / "rtx.h", INC / "rtx_host.h", INC / "rtx_view.h",
            LIB / "librtx_hip.so", LIB / "librtx_host.so"]
    if force or _stale(out, deps):
        _run(["g++", "-std=c++17", "-O2", "-Wall", f"-I{INC}", src, "-o", out, f"-L{LIB}", "-lrtx_hip", "-lrtx_host",
              "-ldl", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"])
    return out


def build_oracle(force: bool = False) -> Path:
    """Test infrastructure: the C restatement used only by tests/, smoke() and bench's
    cpu_baseline leg."""
    bdir = ORACLE / "_build"
    bdir.mkdir(exist_ok=True)
    out = bdir / "librtx_oracle.so"
    src = ORACLE / "rtx_oracle.c"
    if force or _stale(out, [src, INC / "rtx.h"]):
        _run(["gcc", "-std=c11", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
              "-Wall", "-Wextra", f"-I{INC}", src, "-o", out, "-lm", "-lpthread"])
    return out


def build_checkers(force: bool = False) -> Path:
    """Test infrastructure: the brute-force CPU restatement of the cull records
    (tools/cull_records_ref.c), the checker of tests/test_gpu_cull.py."""
    bdir = REPO / "tools" / "bin"
    bdir.mkdir(exist_ok=True)
    out = bdir / "libcull_records_ref.so"
    src = REPO / "tools" / "cull_records_ref.c"
    if force or _stale(out, [src, CSRC / "rtx_cull.h"]):
        _run(["gcc", "-std=c11", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-Wall", "-Wextra",
              src, "-o", out, "-lm"])
    return out


def build_reference(force: bool = False) -> Path | None:
    """Test infrastructure: the reference's own sources compiled in place (oracle/ref)."""
    out = ORACLE / "_ref" / "ref_harness"
    if not (REFERENCE / "source" / "Scene.cpp").exists():
        return out if out.exists() else None
    if force and (ORACLE / "_ref").exists():
        shutil.rmtree(ORACLE / "_ref")
    _run(["make", "-s", "-C", ORACLE / "ref", "-j8"])
    return out


def build_all(force: bool = False) -> None:
    build_host(force)
    build_oracle(force)
    build_checkers(force)
    build_hip(force)
    build_reference(force)   # after librtx_hip.so: oracle/_ref/ref_binding links it
    build_cli(force)
    build_view(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
