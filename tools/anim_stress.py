"""Device Update stress (rtx_anim_*): many chained Updates at random times, each
compared word for word with the host Update (the reference's order), on one context.  The build's
workgroups hand tasks to each other across XCDs inside the launch; a stale line would show as a
mismatch here.  Usage (GPU box): python tools/anim_stress.py [updates] [scene,...]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceAnimation, DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402
from test_gpu_anim import _compare_state  # noqa: E402


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    scenes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["W4_Optional", "W4_Bunny", "W4_Reference"]
    rng = np.random.default_rng(5)
    ctx = DeviceContext(0)
    for name in scenes:
        dev_scene, host_scene = HostScene(name), HostScene(name)
        anim = DeviceAnimation(dev_scene, ctx)
        for i in range(n):
            t = float(rng.uniform(0.0, 20.0))
            anim.update(t, ctx)
            host_scene.update(t)
            anim.status(0)
            for k in range(len(anim.mesh_ids)):
                _compare_state(anim, host_scene, k)
        anim.close()
        print(f"{name}: {n} chained device Updates, every one word-for-word equal to the host's", flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
