"""Source-mode (SAMPLE_SOURCE = true, the reference default) sampler throughput on synthetic data
(bench.source_sampler_leg): B chains x K Philox MH steps with the default operator table, steps/s,
us per step and ESS/s of the log-likelihood traces.  Prints one JSON line.

  python tools/bench_source_sampler.py --sites 100 --features 36 --states 5 --zones 6 --families 6 --chains 128
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sites", type=int, default=100)
    p.add_argument("--features", type=int, default=36)
    p.add_argument("--states", type=int, default=5)
    p.add_argument("--zones", type=int, default=6)
    p.add_argument("--families", type=int, default=6)
    p.add_argument("--chains", type=int, default=128)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--burnin", type=int, default=2000)
    p.add_argument("--seed", type=int, default=3)
    a = p.parse_args()
    import bench
    shape = {k: getattr(a, k) for k in ("sites", "features", "states", "zones", "families")}
    print(json.dumps(bench.source_sampler_leg(shape, a.chains, a.steps, a.burnin, a.seed)))


if __name__ == "__main__":
    main()
