"""Time the reference's own sampler (sbayes ZoneMCMC, one chain, one CPU core) on the Balkan and
South America configs — BUILD CONTAINER ONLY (imports /root/reference through
tests/golden/refenv.py).  Prints MH steps/s per core; the numbers are recorded in DESIGN.md next
to the GPU's (bench.py real-data legs)."""
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import refenv  # noqa: E402


def run(name, n_zones, steps, seed=1):
    from sbayes.experiment_setup import Experiment
    from sbayes.load_data import Data
    from sbayes.mcmc_setup import MCMC
    from sbayes.sampling.zone_sampling import ZoneMCMC
    d = refenv.scratch_copy(f"experiments/{name}")
    cwd = os.getcwd()
    os.chdir(d)
    try:
        with open("config.json") as f:
            raw = json.load(f)
        custom = {"model": {"N_AREAS": n_zones}}
        for low, up in (("features", "FEATURES"), ("feature_states", "FEATURE_STATES")):
            if low in raw.get("data", {}):
                custom.setdefault("data", {})[up] = raw["data"][low]
        if name == "south_america":
            custom.setdefault("data", {})["CRS"] = None
        exp = Experiment(experiment_name="timing", log=False)
        exp.load_config(config_file="config.json", custom_settings=custom)
        data = Data(experiment=exp)
        data.load_features()
        data.load_universal_counts()
        data.load_inheritance_counts()
        mcmc = MCMC(data=data, experiment=exp)
        mc = exp.config["mcmc"]
        np.random.seed(seed)
        random.seed(seed)
        smp = ZoneMCMC(data=data, model=mcmc.model, n_chains=1, operators=mcmc.ops,
                       var_proposal=mc["PROPOSAL_PRECISION"], p_grow_connected=mc["P_GROW_CONNECTED"],
                       initial_size=mc["M_INITIAL"], logger=None)
        t0 = time.perf_counter()
        smp.generate_samples(steps, max(1, steps // 10))
        el = time.perf_counter() - t0
        return {"config": name, "n_zones": n_zones, "steps": steps, "seconds": el,
                "steps_per_sec_per_core": steps / el}
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    refenv.setup()
    for name, z, steps in (("balkan", 3, 2000), ("south_america", 6, 1000)):
        print(json.dumps(run(name, z, steps)), flush=True)
