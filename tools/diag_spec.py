import os, sys
sys.path[:0] = ['/root/repo', '/root/repo/tests']
import numpy as np
import oracle_bind
from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.renderer import DeviceContext
from gp1_raytracer_2223_amd.scene import HostScene, RENDERABLE
a = DeviceContext(0)
os.environ["RTX_NO_SPEC"] = "1"; b = DeviceContext(0); del os.environ["RTX_NO_SPEC"]
order = RENDERABLE
for name in order:
    for t in (-1.0,):
        hs = HostScene(name)
        s, cam = hs.view()
        p = abi.make_params(480, 270)
        a.upload(s); b.upload(s)
        r = oracle_bind.render(s, cam, p)[0]
        for k in range(3):
            apx, _ = a.render(cam, p); bpx, _ = b.render(cam, p)
            print(name, k, "spec!=generic", int((apx != bpx).sum()), "spec!=oracle", int((apx != r).sum()), "generic!=oracle", int((bpx != r).sum()),
                  "split", a.split_info(), b.split_info(), "tune", a.split_tune_info()["factor"], b.split_tune_info()["factor"], flush=True)
