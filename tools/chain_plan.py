#!/usr/bin/env python3
"""Parity record of a candidate conv plan: the bench chain of
tests/test_bench_pipeline_gpu.py (config 3's 8 streams x 160 frames against the oracle chain,
resynced near-ties) on the given plan and frames-per-forward, printing the chain summary.

usage: chain_plan.py <plan.json> [tbatch]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def main():
    import test_bench_pipeline_gpu as T
    from conftest import pkg

    plan = os.path.relpath(os.path.abspath(sys.argv[1]), REPO)
    tb = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    P = pkg()
    chain = T.build_chain([P.shard.stream_seed(s, T.S) for s in range(T.S)], T.F, T.TARGETS)
    out = T.check_chain(chain, plan, tb)
    print("CHAIN_OK", out["near_tie_flips"], out["order_ties"])


if __name__ == "__main__":
    main()
