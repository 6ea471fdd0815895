"""A rank of bench.py's N>1 setup on CPU (gloo), for the failure-bound tests
in test_dist.py: launched by torch.distributed.run, every rank runs bench.py's
own `dist_setup` under `rank_guard`; rank `--fail-rank` misbehaves:

* ``before_init`` — exits (status 0) before joining the process group: the
  other ranks' rendezvous must fail at the deadline;
* ``after_init`` — exits (status 0) after joining, before the first
  collective of the run: the others' collective must fail;
* ``raise`` — raises after joining: the launcher must stop the others.

Rank 0 prints "ok" only if everything succeeded (it never should here)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["before_init", "after_init", "raise"], required=True)
    ap.add_argument("--fail-rank", type=int, default=1)
    ap.add_argument("--timeout", type=float, default=10.0)
    a = ap.parse_args()
    import bench
    from rt_amd.dist import rank_guard

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    with rank_guard(rank, "dist_fail_worker"):
        if rank == a.fail_rank and a.mode == "before_init":
            sys.exit(0)
        dist, seen, _ = bench.dist_setup("gloo", 0, world, a.timeout)
        assert seen == world
        if rank == a.fail_rank:
            if a.mode == "after_init":
                os._exit(0)
            raise RuntimeError("injected failure")
        import torch

        x = torch.ones(1)
        dist.all_reduce(x)  # the peer never joins this one
        dist.barrier()
        print("ok", flush=True)


if __name__ == "__main__":
    main()
