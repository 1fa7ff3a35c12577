import sys
from pathlib import Path
sys.path.insert(0, "/root/repo" if Path("/root/repo/gp1_raytracer_2223_amd").exists() else ".")
from gp1_raytracer_2223_amd import abi
abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext
from gp1_raytracer_2223_amd.scene import HostScene
ctx = DeviceContext(0)
for name in ["W1", "W2", "W3", "W4_Bunny", "W4_Optional", "Synthetic100k", "Bunny8Lights"]:
    for t in (-1.0, 0.7, 2.3):
        try:
            hs = HostScene(name)
        except Exception as e:
            print(name, "skip", e); break
        if t >= 0: hs.update(t)
        s, cam = hs.view()
        ctx.upload(s)
        print(name, t, "parts", ctx.split_info()[1], "cull", ctx.cull_info())
ctx.close()
