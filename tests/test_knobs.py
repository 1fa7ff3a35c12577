"""Every environment knob the native libraries read is in INTEGRATION.md's table (ADVICE / VERDICT r05:
the configuration surface is documented where an integrator looks for it)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "gp1_raytracer_2223_amd" / "csrc"


def test_every_env_knob_is_documented():
    text = (ROOT / "INTEGRATION.md").read_text()
    knobs = set()
    for f in list(SRC.glob("*.hip")) + list(SRC.glob("*.cpp")) + list((SRC / "host").glob("*.cpp")):
        knobs |= set(re.findall(r'getenv\("(RTX_[A-Z0-9_]+)"\)', f.read_text()))
    assert knobs, "no knobs found: the source layout changed"
    missing = sorted(k for k in knobs if k not in text)
    assert not missing, f"undocumented knobs: {missing}"
