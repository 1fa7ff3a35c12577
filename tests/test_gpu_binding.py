"""The boundary pinned to the reference's own types.

oracle/_ref/ref_binding is INTEGRATION.md §2's reference-side binding compiled against
/root/reference/source (the reference's dae::Scene, TriangleMesh, Material classes, built in place
by oracle/ref/Makefile) with static_asserts that include/rtx.h's records are byte-compatible with
dae::Sphere / Plane / BVHNode / Light — the build fails otherwise.  Here it runs: the reference's
Scene_W4_BunnyScene::Initialize(), the Scene flattened by the binding's casts, rtx_upload_scene +
rtx_render on the GPU, and the frame must equal the reference's own frame bit for bit
(tests/golden/config_W4_Bunny_1920x1080.npz, made by the reference's Renderer restatement).
The mesh is re-emitted from our assets as OBJ text (exact float round trip) because
/root/reference does not exist on the GPU box.
"""
import hashlib
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
BINDING = ROOT / "oracle" / "_ref" / "ref_binding"
GOLDEN = ROOT / "tests" / "golden"


def test_binding_built_with_reference_types():
    """CPU: the binding (and its static_asserts) compiled wherever the reference sources exist."""
    if not Path("/root/reference/source/Scene.cpp").exists() and not BINDING.exists():
        pytest.skip("no reference sources and no prebuilt binding")
    assert BINDING.exists(), "oracle/ref/Makefile did not build ref_binding (a static_assert failed?)"


@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,H,exact", [("W4_Bunny", 1920, 1080, True), ("W3", 1280, 720, False)])
def test_reference_scene_through_the_binding(tmp_path, scene, W, H, exact):
    if not BINDING.exists():
        pytest.skip("oracle/_ref/ref_binding not built (needs /root/reference at build time)")
    sys.path.insert(0, str(ROOT))
    from bench import write_obj_from_asset
    from gp1_raytracer_2223_amd import abi
    res = tmp_path / "Resources"
    res.mkdir()
    for a in abi.ASSET_DIR.glob("*.rtxmesh"):
        write_obj_from_asset(a, res / f"{a.stem}.obj")
    out = tmp_path / "frame.bin"
    r = subprocess.run([str(BINDING), str(W), str(H), str(out), scene], cwd=tmp_path, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    px = np.fromfile(out, np.uint32)
    assert px.size == W * H
    g = np.load(GOLDEN / f"config_{scene}_{W}x{H}.npz")
    if exact:
        assert hashlib.sha256(px.tobytes()).hexdigest() == str(g["sha_pixels"][0])
    else:   # powf (Cook-Torrance): the north star's 1 LSB on the reference's samples
        ch = lambda p: np.stack([(p >> 16) & 255, (p >> 8) & 255, p & 255], -1).astype(np.int32)  # noqa: E731
        assert np.abs(ch(px[g["idx"]]) - ch(g["pixels"])).max() <= 1
