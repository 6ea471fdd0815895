"""Markdown rows of DESIGN.md §6 from bench.py logs (one JSON line each).

    python tools/results_table.py gpurun_out/bench_c1.log gpurun_out/bench_c2.log ...
"""
import json
import sys


def row(path):
    d = next(json.loads(l) for l in open(path) if l.startswith('{"metric"'))
    r, fc = d["roofline"], d.get("frame_costs", {})
    cb = d.get("cpu_baseline") or {}
    cba = d.get("cpu_baseline_allcores") or {}
    cam = d.get("camera_buffer") or {}
    tr = r.get("traffic")
    prog = fc.get("progressive") or {}
    fps = prog.get("stream_fps"), prog.get("graph_fps")
    return (f"| {d['config']['workload']} | {d['kernel_ms']} | {d['frame_ms']['median']} | {round(d['value']):,} | "
            f"{r['achieved']} ({r['frac']}) | {cb.get('value', '—')} / {cba.get('value', '—')} | "
            f"{d.get('first_frame_ms', '—')} ms | {d.get('moving_camera_ms_per_frame', '—')} "
            f"({d.get('moving_camera_async_ms', '—')}) | "
            f"{'{:,}'.format(round(fps[0])) if fps[0] else '—'} ({'{:,}'.format(round(fps[1])) if fps[1] else '—'}) | "
            f"{cam.get('build_ms', '—')} ms | {d.get('upload_ms')} ms | "
            f"{round(tr / 1e6, 1) if tr else '—'} |")


if __name__ == "__main__":
    print("| config | kernel ms (mean) | median frame ms | Mray/s | achieved TF (frac of 157.3) | CPU Mray/s 1 core ref / "
          "16 cores port | first frame, warm | moving camera ms/frame sync host (async device) | progressive "
          "frames/s (graph) | camera buffer build | upload | bytes/launch (MB, calibrated) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        print(row(p))
