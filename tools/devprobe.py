"""Device visibility probe for multi-process runs (diagnostic): creates a render context
after each step of bench.py's start-up sequence and reports which step breaks it."""
import ctypes
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
rank = os.environ.get("RANK")
from gp1_raytracer_2223_amd import abi  # noqa: E402

lib = abi.load_hip()


def count(tag):
    h = ctypes.c_void_p()
    rc = lib.rtx_create(ctypes.byref(h), 0)
    why = (lib.rtx_last_error(None) or b"").decode()
    print(f"rank {rank} {tag}: rtx_create rc {rc} {why}", file=sys.stderr, flush=True)
    if rc == 0:
        lib.rtx_destroy(h)


step = int(os.environ.get("PROBE_STEP", "9"))
if step >= 1:
    from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: F401
    from gp1_raytracer_2223_amd.scene import HostScene
    if step == 1:
        count("after package imports")
if step >= 2:
    sys.argv = ["bench.py"]
    import bench
    d = bench.Dist()
    if step == 2:
        count("after Dist")
if step >= 3:
    hs = HostScene("W4_Bunny")
    s, cam = hs.view()
    count("after HostScene")
