"""Host Scene::Update cost (transform + BVH rebuild) per animated scene, for the fast and
the direct BVH builder and several pool sizes.  Each configuration runs in its own
process (the builder and pool size are read once per process).
Usage: python tools/host_update_bench.py [scene ...]"""
import os
import subprocess
import sys

CHILD = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
from gp1_raytracer_2223_amd.scene import HostScene
hs = HostScene(sys.argv[2])
for k in range(50): hs.update(0.01 * k)
n = 400
t0 = time.perf_counter()
for k in range(n): hs.update(0.5 + 0.01 * k)
print(f"{(time.perf_counter() - t0) / n * 1e3:.3f}")
"""
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for scene in sys.argv[1:] or ["W4_Optional", "W4_Bunny"]:
    for label, env in [("direct", {"RTX_HOST_BVH": "direct"}), ("fast x1", {"RTX_HOST_THREADS": "1"}),
                       ("fast x2", {"RTX_HOST_THREADS": "2"}), ("fast x4", {"RTX_HOST_THREADS": "4"}),
                       ("fast x8", {"RTX_HOST_THREADS": "8"}),
                       ("x8 fork>=256", {"RTX_HOST_THREADS": "8", "RTX_HOST_PAR_TRIS": "256"}),
                       ("x8 fork>=128", {"RTX_HOST_THREADS": "8", "RTX_HOST_PAR_TRIS": "128"}),
                       ("x8 fork>=64", {"RTX_HOST_THREADS": "8", "RTX_HOST_PAR_TRIS": "64"}),
                       ("x4 fork>=128", {"RTX_HOST_THREADS": "4", "RTX_HOST_PAR_TRIS": "128"})]:
        e = dict(os.environ)
        e.pop("RTX_HOST_BVH", None)
        e.update(env)
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT, scene], env=e, capture_output=True, text=True, check=True)
        print(f"{scene:12s} {label:13s} update {r.stdout.strip()} ms", flush=True)
