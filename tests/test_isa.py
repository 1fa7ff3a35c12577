"""Code-generation guards for the render kernel (CPU: reads the gfx950 code object in librtx_hip.so).

These pin properties the kernel's speed depends on and that a harmless-looking source change
can silently lose (profiles/r01/ablate_history.md, v6: one side-effecting intrinsic turned every
wave-uniform scene read into a per-lane vector load, +17 % kernel time, with correct output):
  * wave-uniform BVH node pairs and triangles are fetched with one s_load_dwordx16 each,
  * per-lane vector loads are confined to the few per-hit gathers (material, hit record),
  * no scratch, and a VGPR count that keeps >= 7 waves per SIMD.
"""
import os
import re
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
# product variants of the PHASE-0 render kernel (COUNT = false, default-depth stack)
PRODUCT = "_Z17rtx_render_kernelILb0ELi0ELb0E"
DEEP = "_Z17rtx_render_kernelILb0ELi0ELb1E"


def _code_object(tmp_path, lib):
    fb = tmp_path / "fatbin.bin"
    co = tmp_path / "gfx950.co"
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fb)], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"], check=True)
    return co


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    if not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("ROCm LLVM tools not present")
    from gp1_raytracer_2223_amd import build
    lib = os.path.join(os.path.dirname(build.__file__), "lib", "librtx_hip.so")
    if not os.path.exists(lib):
        build.build_hip()
    co = _code_object(tmp_path_factory.mktemp("isa"), lib)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(co)], check=True,
                         capture_output=True, text=True).stdout
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    out = {}
    for m in re.finditer(r"^[0-9a-f]+ <(_Z17rtx_render_kernel\w+)>:", dis, re.M):
        name = m.group(1)
        body = dis[m.end():dis.index("s_endpgm", m.end())]
        meta = {}
        for block in notes.split("  - .")[1:]:
            if re.search(rf"\.name:\s+{name}\b", block):
                for key in ("vgpr_count", "sgpr_count", "private_segment_fixed_size"):
                    mm = re.search(rf"\.{key}:\s+(\d+)", block)
                    if mm:
                        meta[key] = int(mm.group(1))
        out[name] = (body, meta)
    assert any(n.startswith(PRODUCT) for n in out), sorted(out)
    return out


def _product(isa):
    return [(n, b, m) for n, (b, m) in isa.items() if n.startswith(PRODUCT)]


def _spec(name):
    m = re.search(r"ILb0ELi0ELb[01]ELi(\d+)E", name)
    return int(m.group(1)) if m else 0


def test_uniform_records_are_scalar_loads(isa):
    for name, body, _ in _product(isa):
        if _spec(name) & 512:   # kSpecNoMesh: the variant has no BVH / triangle code at all
            continue
        # node pairs + triangles, closest-hit and any-hit, fast and exact slab variants
        assert body.count("s_load_dwordx16") >= 8, f"{name}: 64-byte BVH/triangle records are no longer scalar loads"


def test_vector_loads_only_for_per_lane_gathers(isa):
    for name, body, _ in _product(isa):
        n = len(re.findall(r"\bglobal_load_", body))
        assert n <= 20, f"{name}: {n} vector loads in the render kernel: scene reads fell back to per-lane loads"


def test_registers_and_scratch(isa):
    """No scratch anywhere.  The specialised kernels (every BASELINE config's but W1's) keep >= 7 waves
    per SIMD (<= 72 VGPRs; the one-mesh ones ask for 8); the generic kernel (SPEC = 0: scenes matching
    no variant, W1 / W2 / W3_Test) is built for >= 6 (RTX_MIN_WAVES_PER_EU, <= 80)."""
    for name, _, meta in _product(isa):
        assert meta.get("private_segment_fixed_size") == 0, (name, meta)
        assert meta.get("vgpr_count", 999) <= (72 if _spec(name) else 80), (name, meta)
    deep = [(n, m) for n, (_, m) in isa.items() if n.startswith(DEEP)]
    assert deep and all(m.get("private_segment_fixed_size") == 0 for _, m in deep), deep
