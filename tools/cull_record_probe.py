"""The exact cull's record launches alone (for a rocprofv3 kernel trace): per scene, R rounds of
(upload -> one frame: the box tree, every light's and the camera's records) and (camera moved ->
one frame: that camera's records), each frame synchronised, so the record kernels run without a
concurrent render.  Usage (GPU box): python tools/cull_record_probe.py [R] [scene,...]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402


def main() -> int:
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    scenes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["Synthetic100k", "W4_Optional"]
    for name in scenes:
        ctx = DeviceContext(0)
        hs = HostScene(name)
        s, cam = hs.view()
        p = abi.make_params(256, 144)
        for k in range(R):
            ctx.upload(s)
            ctx.render_async(cam, p)
            ctx.synchronize()
            c = abi.Camera()
            C.memmove(C.byref(c), C.byref(cam), C.sizeof(abi.Camera))
            c.origin[0] = cam.origin[0] + 0.01 * (k + 1)
            ctx.render_async(c, p)
            ctx.synchronize()
        print(name, "cull", ctx.cull_info())
        ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
