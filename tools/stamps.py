"""Per-wave start/end stamps (diagnostic build, RTX_STAMPS=1): occupancy over time, tail,
per-XCD balance.  Usage: RTX_HIP_LIB=.../librtx_hip_stamps.so python tools/stamps.py [scene W H]"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

lib = abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "W4_Bunny"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
lib.rtx_debug_stamps.argtypes = [C.c_void_p, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams),
                                 C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
ctx = DeviceContext(0)
hs = HostScene(name)
s, cam = hs.view()
ctx.upload(s)
# STAMPS_STRIPE=rows,first,step: one rank's share of a striped frame (bench.py's strong scaling)
stripe = [int(x) for x in os.environ.get("STAMPS_STRIPE", "0,0,1").split(",")]
p = abi.make_params(W, H, stripe_rows=stripe[0], stripe_first=stripe[1], stripe_step=stripe[2])
for _ in range(5):
    ctx.time_frames(cam, p, 20)
heavy, nparts = ctx.split_info()
print(f'heavy tiles {heavy}, parts {nparts}')
cap = 8 * ((W + 7) // 8) * ((H + 7) // 8) + 6 * 1024
buf = np.zeros(cap, np.uint64)
nw = C.c_uint64()
abi.check(lib.rtx_debug_stamps(ctx.h, C.byref(cam), C.byref(p), buf.ctypes.data_as(C.POINTER(C.c_uint64)),
                               cap, C.byref(nw)), "stamps", ctx.h)
st = buf[: 8 * nw.value].reshape(-1, 8)
split = buf[8 * nw.value: 8 * nw.value + 6 * 1024].reshape(2, 1024, 3)
wave_id = np.arange(len(st))
keep = st[:, 1] > 0   # heavy tiles' main-kernel waves exit at once (split rendering)
st, wave_id = st[keep], wave_id[keep]
t0 = st[:, 0].min()
start = (st[:, 0] - t0) / 100.0   # s_memrealtime = 100 MHz -> us
end = (st[:, 1] - t0) / 100.0
dur = end - start
xcc = (st[:, 2] >> 32).astype(int)
print(f"{name} {W}x{H}: waves {len(st)}  kernel span {end.max():.1f} us  wave dur mean {dur.mean():.2f} "
      f"p50 {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f} us")
print(f"  sum of wave-us / span = {dur.sum() / end.max():.0f} concurrent waves on average")
for q in (10, 25, 50, 75, 90, 99, 100):
    print(f"  {q:3d}% of waves started by {np.percentile(start, q):7.1f} us, ended by {np.percentile(end, q):7.1f} us")
tt = np.linspace(0, end.max(), 21)
conc = [int(((start <= x) & (end > x)).sum()) for x in tt]
print("  concurrency over time:", conc)
dq = np.percentile(dur, [50, 90, 99, 99.9])
print("  wave duration p50/p90/p99/p99.9 (us):", " / ".join(f"{x:.1f}" for x in dq))
late = end > 0.9 * end.max()
print(f"  waves still running in the last 10% of the span: {int(late.sum())}, of them started in the first 10%: "
      f"{int((late & (start < 0.1 * end.max())).sum())}")
for x in range(8):
    sel = xcc == x
    if sel.any():
        print(f"  xcc {x}: waves {sel.sum()} busy-us {dur[sel].sum():.0f} last end {end[sel].max():.1f}")
nodes = st[:, 3].astype(np.int64)
tris = st[:, 4].astype(np.int64)
lane_slab = (st[:, 5] >> 32).astype(np.int64)
lane_tri = (st[:, 5] & 0xffffffff).astype(np.int64)
print(f"  wave node-pair steps: mean {nodes.mean():.0f} p50 {np.median(nodes):.0f} max {nodes.max()}; "
      f"tri steps: mean {tris.mean():.0f} max {tris.max()}")
tiles_x = (W + 7) // 8
order = np.argsort(-dur)[:12]
prim = st[:, 6] / 100.0
shad = st[:, 7] / 100.0
print("  slowest waves: dur_us  start_us  node_steps  tri_steps  slab_eff  tri_eff  prim_us  shadow_walk_us  rest_us  (px0, py0)")
for w in order:
    ty, tx = divmod(int(wave_id[w]), tiles_x)
    x0 = tx * 8
    y0 = ty * 8
    se = lane_slab[w] / max(1, 128 * nodes[w])
    te = lane_tri[w] / max(1, 64 * tris[w])
    print(f"    {dur[w]:9.1f} {start[w]:9.1f} {nodes[w]:10d} {tris[w]:10d} {se:9.3f} {te:8.3f} {prim[w]:8.1f} "
          f"{shad[w]:15.1f} {dur[w] - prim[w] - shad[w]:8.1f}  ({x0}, {y0})")
us_per_step = dur / np.maximum(1, nodes + tris)
print(f"  us per (node+tri) step: p50 {np.median(us_per_step):.3f}  slowest-wave {us_per_step[order[0]]:.3f}")
for ph in range(2):
    sp = split[ph, :nparts]
    if sp[:, 0].sum() == 0:
        continue
    tot = sp[:, 0] / 100.0
    mx = sp[:, 1] / 100.0
    print(f"  split phase {ph + 1}: wave-us total {tot.sum():.0f}, per part mean {tot.mean():.0f} max {tot.max():.0f}; "
          f"slowest wave {mx.max():.1f} us (part {int(mx.argmax())}); steps total {int(sp[:, 2].sum())}")
    top = np.argsort(-tot)[:6]
    print("    heaviest parts (part: wave-us, max wave us, steps):",
          ", ".join(f"{int(k)}: {tot[k]:.0f}/{mx[k]:.0f}/{int(sp[k, 2])}" for k in top))
