"""Convert the reference's OBJ resources into the pre-tokenised .rtxmesh assets the
host scene layer loads (positions + indices exactly as our ParseOBJ restatement reads
them; normals are recomputed at load time the way Utils::ParseOBJ does).

Run in the build container (needs /root/reference):  python tools/make_assets.py
"""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gp1_raytracer_2223_amd import abi  # noqa: E402
from gp1_raytracer_2223_amd.build import build_host  # noqa: E402

RES = Path("/root/reference/source/Resources")
STEMS = ["lowpoly_bunny2", "Assignment3D1", "simple_object", "simple_cube", "simple_quad"]

if __name__ == "__main__":
    build_host()
    lib = abi.load_host()
    abi.ASSET_DIR.mkdir(exist_ok=True)
    for stem in STEMS:
        out = abi.ASSET_DIR / f"{stem}.rtxmesh"
        rc = lib.rtx_host_obj_to_asset(str(RES / f"{stem}.obj").encode(), str(out).encode())
        abi.check(rc, f"convert {stem}")
        print(out, out.stat().st_size)
