"""The C-ABI boundary: struct layouts agree between include/rtx.h (C compiler) and the
ctypes mirror, every entry point the headers declare is exported, the reference-layout
records really are byte-compatible with the reference's structs, and the product
library does not link the oracle."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from gp1_raytracer_2223_amd import abi

ROOT = Path(__file__).resolve().parents[1]
INC = ROOT / "include"

STRUCTS = {
    "rtx_sphere": (abi.Sphere, ["origin", "radius", "material"]),
    "rtx_plane": (abi.Plane, ["origin", "normal", "material"]),
    "rtx_bvh_node": (abi.BVHNode, ["min", "max", "first_idx", "idx_count", "left_node"]),
    "rtx_mesh": (abi.Mesh, ["positions", "n_positions", "indices", "n_indices", "normals", "nodes", "n_nodes",
                            "cull_mode", "material"]),
    "rtx_light": (abi.Light, ["origin", "direction", "color", "intensity", "type"]),
    "rtx_material": (abi.Material, ["kind", "color", "kd", "ks", "exponent", "metalness", "roughness"]),
    "rtx_scene": (abi.Scene, ["spheres", "n_spheres", "planes", "n_planes", "meshes", "n_meshes", "lights",
                              "n_lights", "materials", "n_materials"]),
    "rtx_camera": (abi.Camera, ["origin", "right", "up", "forward", "fov"]),
    "rtx_pixel_format": (abi.PixelFormat, ["rshift", "gshift", "bshift", "amask"]),
    "rtx_render_params": (abi.RenderParams, ["width", "height", "lighting_mode", "shadows_enabled", "format",
                                             "stripe_rows", "stripe_first", "stripe_step"]),
}


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rtx.h"', '#include "rtx_host.h"',
             "int main(void) {"]
    for s, (_, fields) in STRUCTS.items():
        lines.append(f'printf("{s} size %zu\\n", sizeof({s}));')
        for f in fields:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0; }")
    (d / "l.c").write_text("\n".join(lines))
    subprocess.run(["gcc", "-std=c11", f"-I{INC}", str(d / "l.c"), "-o", str(d / "l")], check=True)
    out = subprocess.run([str(d / "l")], check=True, capture_output=True, text=True).stdout
    return dict(line.rsplit(" ", 1) for line in out.strip().splitlines())


@pytest.mark.parametrize("name", list(STRUCTS))
def test_struct_layout(c_layout, name):
    cls, fields = STRUCTS[name]
    assert int(c_layout[f"{name} size"]) == C.sizeof(cls)
    for f in fields:
        assert int(c_layout[f"{name}.{f}"]) == getattr(cls, f).offset, f


def test_reference_record_sizes():
    # dae::Sphere / Plane / BVHNode / Light sizes on x64 (DataTypes.h:13-54, 528-536)
    assert C.sizeof(abi.Sphere) == 20 and C.sizeof(abi.Plane) == 28
    assert C.sizeof(abi.BVHNode) == 36 and C.sizeof(abi.Light) == 44


def _declared(header: Path) -> list[str]:
    txt = header.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*|rtx_ctx\*)\s+(rtx_\w+)\s*\(", txt, re.M)))


def test_hip_library_exports_every_declared_symbol():
    lib = abi.load_hip()   # loads without a GPU; no compute call is made here
    names = _declared(INC / "rtx.h") + _declared(INC / "rtx_diag.h")
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(abi.HIP_SYMBOLS), set(names) - set(abi.HIP_SYMBOLS)


def test_host_library_exports_every_declared_symbol():
    lib = abi.load_host()
    for n in _declared(INC / "rtx_host.h") + _declared(INC / "rtx_view.h"):
        assert hasattr(lib, n), n


def test_product_header_has_no_diagnostics():
    """rtx.h is the product boundary (render, group, device Update, gather); timing, counters and the
    scheduler's internals live in rtx_diag.h."""
    prod = set(_declared(INC / "rtx.h"))
    diag = set(_declared(INC / "rtx_diag.h"))
    assert not prod & diag
    for n in ("rtx_time_views", "rtx_count_work", "rtx_split_info", "rtx_cull_dump", "rtx_schedule_state",
              "rtx_anim_stamps", "rtx_light_major_info", "rtx_inflight_info"):
        assert n in diag and n not in prod, n
    for n in ("rtx_create", "rtx_upload_scene", "rtx_render", "rtx_last_error", "rtx_destroy", "rtx_gather_async",
              "rtx_group_render", "rtx_anim_update"):
        assert n in prod, n


def test_product_does_not_link_oracle():
    for so in (abi.LIB_DIR / "librtx_hip.so", abi.LIB_DIR / "librtx_host.so"):
        out = subprocess.run(["readelf", "-d", str(so)], check=True, capture_output=True, text=True).stdout
        assert "oracle" not in out and "ref_harness" not in out
        assert b"rtx_oracle" not in so.read_bytes()


def test_abi_version():
    assert abi.load_hip().rtx_abi_version() == 2   # 2: diagnostics moved to rtx_diag.h (same symbols)


def test_create_reports_why_it_failed():
    """Bad arguments come back as codes, never as a crash; a failed rtx_create leaves its
    reason for rtx_last_error(NULL).  (No GPU here: the device query itself fails or the
    device id is out of range — either way a reason is recorded.)"""
    lib = abi.load_hip()
    assert lib.rtx_create(None, 0) == abi.RTX_E_INVALID
    h = C.c_void_p()
    rc = lib.rtx_create(C.byref(h), 1 << 20)   # no machine has that many devices
    assert rc in (abi.RTX_E_DEVICE, abi.RTX_E_INVALID)
    assert not h.value
    assert lib.rtx_last_error(None)   # non-empty reason
