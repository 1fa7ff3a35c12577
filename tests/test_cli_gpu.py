"""The headless C++ host program (lib/rtx_render): screenshot and the reference's F6
benchmark mode (Timer.cpp:44-131: one-second dFPS windows -> benchmark.txt)."""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_bind
from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.scene import HostScene

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "gp1_raytracer_2223_amd" / "lib" / "rtx_render"
pytestmark = pytest.mark.gpu


def _bmp_pixels(path: Path, W: int, H: int) -> np.ndarray:
    b = path.read_bytes()
    assert b[:2] == b"BM" and int.from_bytes(b[10:14], "little") == 54
    rows = np.frombuffer(b, np.uint32, W * H, 54).reshape(H, W)
    return rows[::-1].reshape(-1)   # bottom-up


def test_screenshot_matches_oracle(tmp_path):
    if not EXE.exists():
        pytest.skip("rtx_render not built")
    W, H = 160, 120
    out = tmp_path / "shot.bmp"
    subprocess.run([str(EXE), "W4_Bunny", str(W), str(H), "--out", str(out)], check=True, cwd=tmp_path, timeout=120)
    hs = HostScene("W4_Bunny")
    s, cam = hs.view()
    ref, _ = oracle_bind.render(s, cam, abi.make_params(W, H))
    assert np.array_equal(_bmp_pixels(out, W, H), ref)


def test_benchmark_mode_writes_reference_format(tmp_path):
    if not EXE.exists():
        pytest.skip("rtx_render not built")
    r = subprocess.run([str(EXE), "W4_Bunny", "320", "240", "--benchmark", "2"], check=True, cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert "**BENCHMARK STARTED**" in r.stdout and "**BENCHMARK FINISHED**" in r.stdout
    lines = (tmp_path / "benchmark.txt").read_text().splitlines()
    assert [l.split(" = ")[0] for l in lines] == ["FRAMES", "HIGH", "LOW", "AVG"]
    vals = {l.split(" = ")[0]: float(l.split(" = ")[1]) for l in lines}
    assert vals["FRAMES"] == 2 and vals["LOW"] <= vals["AVG"] <= vals["HIGH"] and vals["LOW"] > 0
    m = re.search(r"frames (\d+) \(animated\)", r.stdout)
    assert m and int(m.group(1)) >= 2


def _channels(px: np.ndarray) -> np.ndarray:
    return np.stack([(px >> s) & 0xFF for s in (16, 8, 0)], -1).astype(np.int32)


@pytest.mark.parametrize("scene,inflight,exact,device", [("W4_Bunny", 2, True, False), ("W4_Optional", 2, False, False),
                                                         ("W4_Optional", 3, False, False),
                                                         ("W4_Optional", 4, False, False),
                                                         ("W4_Reference", 1, False, False),
                                                         ("W4_Bunny", 2, True, True), ("W4_Optional", 3, False, True),
                                                         ("W4_Reference", 2, False, True)])
def test_pipelined_frame_loop_matches_oracle(tmp_path, scene, inflight, exact, device):
    """The overlapped frame loop (frame k+1's Update and BVH rebuild on the host while frame
    k renders on another context) renders every frame of an animated sequence exactly as
    the reference's serial loop: Update(t_k) on one persistent scene, then Render.  With 2+
    frames in flight the host Updates themselves run ahead on worker threads, each into its
    own copy of the scene (1 or 2 of them: inflight 2 / 3-4).  With --device-update the Update
    itself runs on the device (rtx_anim_*)."""
    if not EXE.exists():
        pytest.skip("rtx_render not built")
    W, H = 160, 120
    times = [0.3, 0.9, 1.7, 2.2, 3.1]
    subprocess.run([str(EXE), scene, str(W), str(H), "--sequence", ",".join(map(str, times)), "--inflight",
                    str(inflight), "--out", str(tmp_path / "f.bmp")] + (["--device-update"] if device else []),
                   check=True, cwd=tmp_path, timeout=120)
    hs = HostScene(scene)
    for k, t in enumerate(times):
        hs.update(t)
        s, cam = hs.view()
        ref, _ = oracle_bind.render(s, cam, abi.make_params(W, H))
        got = _bmp_pixels(tmp_path / f"f_{k}.bmp", W, H)
        if exact:
            assert np.array_equal(got, ref), f"frame {k}: {int((got != ref).sum())} pixels differ"
        else:   # powf (Phong) is the device libm's: the north star's 1-LSB bound
            assert int(np.abs(_channels(got) - _channels(ref)).max()) <= 1, f"frame {k}"


def test_viewer_keys_headless(tmp_path):
    """The viewer's frame loop (lib/rtx_view, csrc/cli/rtx_view.cpp) with a scripted key sequence and no
    window: F3 F3 (Combined -> ObservedArea -> Radiance), F2 (shadows off), X (screenshot of that
    frame), F6 (benchmark started), then one more frame.  Each frame's state is printed, and the
    screenshot is the oracle's frame in the state the keys left (main.cpp:63-107)."""
    view = ROOT / "gp1_raytracer_2223_amd" / "lib" / "rtx_view"
    if not view.exists():
        pytest.skip("rtx_view not built")
    W, H = 160, 120
    r = subprocess.run([str(view), "W3", str(W), str(H), "--keys", "F3,F3,F2,X,F6", "--out", "shot.bmp"], check=True,
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    states = re.findall(r"frame (\d+): mode (\d) shadows (\d)", r.stdout)
    assert states == [("0", "0", "1"), ("1", "1", "1"), ("2", "1", "0"), ("3", "1", "0"), ("4", "1", "0"),
                      ("5", "1", "0")], r.stdout
    assert "Screenshot saved!" in r.stdout and "**BENCHMARK STARTED**" in r.stdout
    hs = HostScene("W3")
    s, cam = hs.view()
    ref, _ = oracle_bind.render(s, cam, abi.make_params(W, H, mode=1, shadows=False))   # Radiance: no powf
    assert np.array_equal(_bmp_pixels(tmp_path / "shot.bmp", W, H), ref)
