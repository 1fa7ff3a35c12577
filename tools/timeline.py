"""Print the last frames' kernel timeline from rocprofv3 --kernel-trace CSVs (render kernels only):
start / end / duration in us from the first printed dispatch, the queue, and the phase (main = PHASE 0
on the frame stream, P1-P3 = the split chain on its own stream).
Usage: python tools/timeline.py <trace dir> [label] [n dispatches]"""
import csv
import sys
from pathlib import Path


def main() -> None:
    d = Path(sys.argv[1])
    label = sys.argv[2] if len(sys.argv) > 2 else d.name
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 48
    f = next(d.glob("*kernel_trace.csv"))
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rend = [r for r in rows if "rtx_render_kernel" in r["Kernel_Name"]][-n:]
    t0 = int(rend[0]["Start_Timestamp"])
    print(f"== {label}")
    for r in rend:
        phase = r["Kernel_Name"].split("<")[1].split(",")[1].strip()
        name = {"0": "main", "1": "P1", "2": "P2", "3": "P3"}.get(phase, "PHASE " + phase)
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1000:9.1f} {e / 1000:9.1f} {(e - s) / 1000:8.1f} q{r.get('Queue_Id', '?')} {name}")


if __name__ == "__main__":
    main()
