"""Frame-tail estimate from a per-tile cost map (tools/prof_tiles.py --out).

Greedy list scheduling of the frame's one-wave workgroups onto the chip's
wave slots (CUs x SIMDs x waves per SIMD), in a given dispatch order: each
next tile starts on the slot that frees first.  Prints the makespan against
the ideal (summed wave time / slots) for the hardware's row-major order,
heavy-tiles-first, and a few others — how much of a frame the ramp-down
costs, and how much an order could win back, before any kernel is written.

    python tools/tail_sim.py gpurun_out/tiles_c2.npz --waves 7
"""
import argparse
import heapq
import json

import numpy as np


def makespan(costs, slots):
    h = [0.0] * min(slots, len(costs))
    heapq.heapify(h)
    end = 0.0
    for c in costs:
        t = heapq.heappop(h) + float(c)
        end = max(end, t)
        heapq.heappush(h, t)
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--simds", type=int, default=4)
    ap.add_argument("--waves", type=int, default=7)
    a = ap.parse_args()
    z = np.load(a.npz)
    tot, valid = z["tot"].astype(np.float64), z["valid"]
    rows = np.where(valid.any(axis=1))[0]
    cols = np.where(valid.any(axis=0))[0]
    grid = tot[: rows.max() + 1, : cols.max() + 1]
    slots = a.cus * a.simds * a.waves
    ideal = grid.sum() / slots
    orders = {
        "row_major": grid.reshape(-1),
        "heavy_first": np.sort(grid.reshape(-1))[::-1],
        "light_first": np.sort(grid.reshape(-1)),
        "rows_reversed": grid[::-1].reshape(-1),
    }
    res = {"tiles": int(grid.size), "slots": slots, "mean_wave_clk": float(grid.mean()),
           "ideal_clk": ideal}
    for k, v in orders.items():
        m = makespan(v, slots)
        res[k] = {"makespan_clk": round(m), "vs_ideal": round(m / ideal, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
