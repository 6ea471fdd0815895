"""tools/tail_sim.py: the list-scheduling model behind the dispatch-order
experiment (profiles/r02/s26_order)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from tail_sim import makespan  # noqa: E402


def test_makespan_equal_costs_fill_generations():
    # 10 unit tiles on 4 slots: three generations, the last half full
    assert makespan([1.0] * 10, 4) == 3.0
    assert makespan([1.0] * 8, 4) == 2.0


def test_makespan_heavy_first_beats_heavy_last():
    light, heavy = [1.0] * 12, [4.0]
    assert makespan(heavy + light, 4) == 4.0
    assert makespan(light + heavy, 4) == 7.0


def test_makespan_fewer_tiles_than_slots():
    assert makespan([2.0, 5.0, 1.0], 8) == 5.0
