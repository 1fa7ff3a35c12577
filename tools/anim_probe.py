"""Device-side Update probe: frames of the device-built scene vs the host upload, per render
path switch, and the Update's device time.  Usage (GPU box): python tools/anim_probe.py [scene]"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceAnimation, DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "W4_Reference"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (480, 270)
dev, host = HostScene(name), HostScene(name)
a, b = DeviceContext(0), DeviceContext(0)
anim = DeviceAnimation(dev, a)
p = abi.make_params(W, H)
s, cam = host.view()
b.upload(s)
for mode in (3, 0):
    p.lighting_mode = mode
    apx, _ = a.render(cam, p)
    bpx, _ = b.render(cam, p)
    print(f"registration image, mode {mode}: {(apx != bpx).sum()} px differ, nonzero {np.count_nonzero(apx)}/{np.count_nonzero(bpx)}")
p.lighting_mode = 3
for t in (1.3, 2.7):
    anim.update(t, a)
    host.update(t)
    s, cam = host.view()
    b.upload(s)
    print("status", anim.status(0))
    for k in range(3):
        apx, _ = a.render(cam, p)
        bpx, _ = b.render(cam, p)
        print(f"t={t} frame {k}: {(apx != bpx).sum()} px differ, nonzero {np.count_nonzero(apx)}/{np.count_nonzero(bpx)}")
# device Update cost: back-to-back updates on one context
a.synchronize()
for n in (1, 50):
    t0 = time.perf_counter()
    for i in range(n):
        anim.update(0.01 * i, a)
    anim.status(0)
    dt = (time.perf_counter() - t0) / n
    print(f"{name}: {n} device Updates: {dt * 1e3:.3f} ms each (host enqueue + device, serialized)")
t0 = time.perf_counter()
for i in range(50):
    host.update(0.01 * i)
print(f"{name}: host Update {(time.perf_counter() - t0) / 50 * 1e3:.3f} ms each")

# scene image of the device Update vs the registration (host-built) image of the same state
import ctypes as C  # noqa: E402
lib = abi.load_hip()


def image(ctx):
    n = C.c_size_t()
    abi.check(lib.rtx_scene_image(ctx.h, None, 0, C.byref(n)), "rtx_scene_image")
    buf = np.zeros(n.value // 4, np.uint32)
    abi.check(lib.rtx_scene_image(ctx.h, buf.ctypes.data, n.value, C.byref(n)), "rtx_scene_image")
    return buf


d2, h2 = HostScene(name), HostScene(name)
c1, c2 = DeviceContext(0), DeviceContext(0)
an1 = DeviceAnimation(d2, c1)
an1.update(1.3, c1)
h2.update(1.3)
an2 = DeviceAnimation(h2, c2)
i1, i2 = image(c1), image(c2)
diff = np.nonzero(i1 != i2)[0]
print(f"image words {len(i1)} / {len(i2)}, differing words {len(diff)}")
if len(diff):
    runs = np.split(diff, np.nonzero(np.diff(diff) > 1)[0] + 1)
    for r in runs[:12]:
        print(f"  words {r[0]}..{r[-1]} (byte {4 * r[0]}): dev {i1[r[0]:r[0] + 8]} host {i2[r[0]:r[0] + 8]}")

st = (C.c_uint32 * 128)()
abi.check(lib.rtx_anim_stamps(an1.h, 0, st), "rtx_anim_stamps")
w = [int(x) for x in st]


def us(x, ref=None):
    """A stamp (low 32 bits of s_memrealtime, 100 MHz) in us from `ref` (default: the build's start,
    w[8]), as a SIGNED 32-bit difference, so a stamp taken before the start (a worker workgroup
    that entered early) reads negative instead of wrapping to ~42.9 s; an unwritten stamp is None."""
    if x == 0:
        return None
    d = (x - (w[8] if ref is None else ref)) & 0xffffffff
    return (d - (1 << 32) if d >= 1 << 31 else d) / 100.0


def r1(x):
    return None if x is None else round(x, 1)


print(f"status: err {w[0]} deepest {w[1]} nodesUsed {w[2]} parts {w[3]} subtrees {w[4]} task-split ids {w[5]} "
      f"nodes split as tasks {w[6]}")
print(f"build phases (us from start): set-up {r1(us(w[9]))}, root split {r1(us(w[10]))}, "
      f"subtrees {r1(us(w[11]))} .. {r1(us(w[12]))}, output start {r1(us(w[13]))}, ranks {r1(us(w[14]))}, "
      f"frontier {r1(us(w[15]))}")
print(f"subtree 0: staged {r1(us(w[29]))}, levels end {[r1(us(x)) for x in w[32:40] if x]}, levels done {r1(us(w[30]))}, "
      f"ranks {r1(us(w[31]))}")
print(f"output wg0: records written {r1(us(w[57]))}")
if w[61] != w[60] and w[31] != w[29]:
    print(f"shader clock during subtree 0: {((w[61] - w[60]) & 0xffffffff) / (((w[31] - w[29]) & 0xffffffff) / 100.0):.0f} MHz")
print("first splits (size, start, end us):", [(w[16 + k], r1(us(w[20 + 2 * k])), r1(us(w[21 + 2 * k])))
                                               for k in range(min(4, w[6]))])
if w[63]:
    print("top root steps (us from its start):", [r1(us(w[64 + i], w[63])) for i in range(9)])
if w[40]:
    print("subtree-0 root steps (us from its start):", [r1(us(w[41 + i], w[40])) for i in range(9)],
          "bins/axis:", [r1(us(w[50 + a], w[40])) for a in range(3)],
          "sweep lanes done, key reduced:", [r1(us(w[55 + a], w[40])) for a in range(2)],
          "child bounds loop done, reduced:", [r1(us(w[53 + a], w[40])) for a in range(2)])
print("subtrees (start, end us):", [(r1(us(w[80 + 2 * f])), r1(us(w[81 + 2 * f]))) for f in range(min(8, w[4]))])
print("worker workgroup entry (us):", [r1(us(w[112 + f])) for f in range(16)])
print("subtree sizes:", [w[96 + f] for f in range(min(16, w[4]))])
if w[63]:
    print("top root bins per axis done (us from its start):", [r1(us(w[73 + a], w[63])) for a in range(3)])
