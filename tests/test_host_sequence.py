"""Animated frame loops on the host scene layer: after a SEQUENCE of Scene::Update calls
the world geometry, the BVH node array and the triangle permutation still equal the
reference's (tests/golden/seq_*.npz, made by tests/golden/make_seq_goldens.py from the
reference built in place).  Each rebuild permutes the triangles in place
(source/DataTypes.h:335-363), so build k depends on every earlier one; the single-Update
goldens cannot see a divergence that appears only after several rebuilds.

Both BVH builders are checked: the default fast one (SIMD passes over a permutation
array, subtrees on a thread pool) and the direct restatement (RTX_HOST_BVH=direct)."""
import hashlib
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

G = Path(__file__).resolve().parent / "golden"
ROOT = G.parents[1]


def _digest(m: dict) -> str:
    links = m["node_links"].reshape(-1, 3).copy()
    links[links[:, 1] != 0, 2] = 0   # a leaf's leftNode is stale in the reference
    h = hashlib.sha256()
    for a in (m["tpositions"], m["indices"], m["tnormals"], m["node_bounds"], links):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _scene_name(stem: str) -> str:
    return "file:" + str(ROOT / "scenes" / (stem[5:] + ".rtxscene")) if stem.startswith("file_") else stem


_CHILD = r"""
import sys, json
sys.path.insert(0, sys.argv[1])
import numpy as np
from gp1_raytracer_2223_amd.scene import HostScene
name, times, checkpoints = sys.argv[2], json.loads(sys.argv[3]), json.loads(sys.argv[4])
sys.path.insert(0, sys.argv[1] + '/tests')
from test_host_sequence import _digest
out = {}
for n in checkpoints:
    hs = HostScene(name)
    for t in times[:n]:
        hs.update(t)
    out[str(n)] = [_digest(m) for m in hs.arrays()["meshes"]]
print(json.dumps(out))
"""


@pytest.mark.parametrize("builder", ["fast", "direct"])
@pytest.mark.parametrize("path", sorted(G.glob("seq_*.npz")), ids=lambda p: p.stem)
def test_update_sequence_matches_reference(path, builder):
    import json
    g = np.load(path)
    times = [float(t) for t in g["times"]]
    cps = [int(c) for c in g["checkpoints"]]
    env = dict(os.environ)
    if builder == "direct":
        env["RTX_HOST_BVH"] = "direct"
    else:
        env.pop("RTX_HOST_BVH", None)
    # own process: the builder is chosen once per process (environment read at load)
    r = subprocess.run([sys.executable, "-c", _CHILD, str(ROOT), _scene_name(path.stem[4:]), json.dumps(times),
                        json.dumps(cps)], capture_output=True, text=True, env=env, check=True)
    got = json.loads(r.stdout.strip().splitlines()[-1])
    for n in cps:
        assert got[str(n)] == [str(x) for x in g[f"after{n}"]], f"after {n} updates"


def test_nan_mesh_takes_direct_builder(tmp_path):
    """A mesh with NaN coordinates (here a NaN scale) cannot use the fast builder's
    min/max shortcuts (a NaN vertex drops out of min(min(v0, v1), v2) differently from the
    reference's vertex-by-vertex Grow); it must fall back to the direct restatement, so both
    settings give the same arrays."""
    import json
    f = tmp_path / "nan.rtxscene"
    f.write_text("camera 0 2 -8 45\nmaterial lambert 1 1 1 1\nplane 0 0 0 0 1 0 1\n"
                 "mesh lowpoly_bunny2 1 back scale nan 1 1 spin\n"
                 "mesh simple_cube 1 front translate 1 1 0 spin\nlight point 0 5 -4 50 1 1 1\n")
    out = {}
    for builder in ("fast", "direct"):
        env = dict(os.environ)
        env.pop("RTX_HOST_BVH", None)
        if builder == "direct":
            env["RTX_HOST_BVH"] = "direct"
        r = subprocess.run([sys.executable, "-c", _CHILD, str(ROOT), "file:" + str(f), json.dumps([0.4, 1.1, 2.5]),
                            json.dumps([1, 3])], capture_output=True, text=True, env=env, check=True)
        out[builder] = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["fast"] == out["direct"]


@pytest.mark.parametrize("scene", ["W4_Bunny", "W4_Optional"])
def test_pipelined_loop_keeps_one_update_history(scene):
    """The CLI's pipelined frame loop (csrc/cli/rtx_render.cpp, ChainUpdater) updates ONE scene
    serially and uploads snapshots of it (rtx_host_scene_copy_state).  Every snapshot equals a
    scene updated serially through the same times — indices, normals and nodes included, which the
    in-place BVH permutation makes depend on the whole history.  Handing the Updates round robin to
    several scenes (round 5's loop) does not: a scene that skipped an Update keeps another triangle
    order."""
    from gp1_raytracer_2223_amd.scene import HostScene
    times = [0.3, 0.9, 1.7, 2.2]
    serial, chain = HostScene(scene), HostScene(scene)
    snaps = [HostScene(scene), HostScene(scene)]
    for k, t in enumerate(times):
        serial.update(t)
        chain.update(t)
        snap = snaps[k % 2]
        snap.copy_state(chain)
        assert [_digest(m) for m in snap.arrays()["meshes"]] == [_digest(m) for m in serial.arrays()["meshes"]], k
    # round robin over two scenes: the second one never sees Update 0.3
    skipped = HostScene(scene)
    for t in times[1::2]:
        skipped.update(t)
    a, b = serial.arrays()["meshes"][0], skipped.arrays()["meshes"][0]
    assert np.array_equal(a["tpositions"], b["tpositions"])
    assert not np.array_equal(a["indices"], b["indices"])


def test_copy_state_refuses_another_scene():
    from gp1_raytracer_2223_amd.scene import HostScene
    with pytest.raises(Exception):
        HostScene("W4_Bunny").copy_state(HostScene("W4_Optional"))
