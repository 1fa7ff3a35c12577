"""Golden hashes for animated frame loops: the reference's flattened scene after a SEQUENCE
of Scene::Update calls (test infrastructure).

The reference rebuilds every animated mesh's BVH in place at each Update
(source/DataTypes.h:210-236, 294-372): the partition permutes indices / normals /
transformedNormals, so the triangle order of build k depends on every earlier build.  The
single-Update goldens (make_goldens.py, t = 1.3 after Initialize) cannot see a divergence
that only shows after several rebuilds; these can.  Written by the reference built in place
(oracle/_ref/ref_harness, `scene <name> t1,t2,...`), one SHA-256 per mesh array after each
prefix of the sequence.

Usage:  python tests/golden/make_seq_goldens.py
"""
from __future__ import annotations

import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from make_goldens import run  # noqa: E402

# the animated catalogue scenes; Bunny8Lights moves the same mesh as W4_Bunny
SCENES = ["W4_Bunny", "W4_Optional", "W4_Reference", "file:" + str(HERE.parents[1] / "scenes" / "gallery.rtxscene")]
TIMES = [round(0.37 + 0.61 * k, 2) for k in range(16)]
CHECKPOINTS = [1, 2, 5, 16]


def mesh_digest(d: dict, i: int) -> str:
    """SHA-256 over one mesh's world positions, permuted indices and normals, and the
    used BVH nodes (bounds, first/count, and leftNode of inner nodes only: a leaf's
    leftNode is whatever an earlier build left in that slot)."""
    p = f"mesh{i}_"
    links = d[p + "node_links"].reshape(-1, 3).copy()
    links[links[:, 1] != 0, 2] = 0
    h = hashlib.sha256()
    for a in (d[p + "tpositions"], d[p + "indices"], d[p + "tnormals"], d[p + "node_bounds"], links):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main() -> None:
    for name in SCENES:
        out = {"times": np.array(TIMES, np.float32), "checkpoints": np.array(CHECKPOINTS, np.int32)}
        for n in CHECKPOINTS:
            d = run("scene", name, ",".join(f"{t:g}" for t in TIMES[:n]))
            nm = len(d["meshes"]) // 5
            out[f"after{n}"] = np.array([mesh_digest(d, i) for i in range(nm)])
        stem = name if not name.startswith("file:") else "file_" + Path(name[5:]).stem
        np.savez_compressed(HERE / f"seq_{stem}.npz", **out)
        print("seq", stem, flush=True)


if __name__ == "__main__":
    main()
