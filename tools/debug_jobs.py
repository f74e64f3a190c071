"""Debug: the South America K sweep as 1 rank sequential vs 2 ranks job-sharded (sequential /
concurrent); prints the first differing lines of each differing results file."""
import filecmp, json, os, socket, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "tests", "golden", "io", "data", "experiments", "south_america", "config.json")


def port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def run(out, ranks, extra):
    st = {"model": {"N_AREAS": [1, 2, 3, 4, 5, 6], "SAMPLE_SOURCE": True},
          "mcmc": {"N_STEPS": 3000, "N_SAMPLES": 30, "N_CHAINS": 5,
                   "WARM_UP": {"N_WARM_UP_STEPS": 600, "N_WARM_UP_CHAINS": 7}},
          "results": {"RESULTS_PATH": out}}
    args = ["-m", "contact_zones_amd", CFG, "--seed", "11", "--name", "x", "--set", json.dumps(st)] + extra
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if ranks > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(ranks),
               "--master-addr", "127.0.0.1", "--master-port", str(port())] + args
        env["SBZ_DIST_BACKEND"] = "gloo"
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        print(r.stderr[-2000:]); sys.exit(1)
    return sorted(os.path.relpath(os.path.join(d, f), out) for d, _, fs in os.walk(out) for f in fs)


tmp = tempfile.mkdtemp()
base = os.path.join(tmp, "seq")
fb = run(base, 1, ["--jobs", "sequential"])
for name, ranks, extra in (("seq2", 1, ["--jobs", "sequential"]), ("sh_seq", 2, ["--shard", "jobs", "--jobs", "sequential"]),
                           ("sh_con", 2, ["--shard", "jobs"]), ("con", 1, [])):
    o = os.path.join(tmp, name)
    fo = run(o, ranks, extra)
    bad = [f for f in fb if f not in fo or not filecmp.cmp(os.path.join(base, f), os.path.join(o, f), shallow=False)]
    print(name, "differs:", bad)
    for f in bad[:2]:
        a = open(os.path.join(base, f)).read().splitlines()
        b = open(os.path.join(o, f)).read().splitlines()
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                print("  ", f, "line", i, "\n    ", x[:160], "\n    ", y[:160])
                break
