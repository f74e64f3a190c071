"""Import the read-only reference (sBayes) for golden-vector capture — BUILD CONTAINER ONLY.

The reference never travels to the GPU box; nothing in the `-m gpu` tests, smoke()
or bench.py imports this module.  It is used only by the capture scripts in this
directory, which write the small .npz fixtures that do travel.

Three third-party modules the reference imports at module level are absent from
this image and are used only off the hot path:
  fastcluster (sbayes/util.py:23, plotting only), pyproj (sbayes/load_data.py:6,
  sbayes/preprocessing.py:11, CRS only), pycldf (sbayes/experiment_setup.py:20).
Empty stand-in modules with those names are written to a temp dir and put on
sys.path ahead of the reference; bytecode writing is disabled so nothing is
written under /root/reference.
"""
import os
import shutil
import sys
import tempfile

REFERENCE = os.environ.get("SBZ_REFERENCE", "/root/reference")


def setup():
    if not os.path.isdir(os.path.join(REFERENCE, "sbayes")):
        raise RuntimeError(f"reference not found at {REFERENCE} (capture runs in the build container only)")
    sys.dont_write_bytecode = True
    stub_dir = tempfile.mkdtemp(prefix="sbz_refstubs_")
    with open(os.path.join(stub_dir, "fastcluster.py"), "w") as f:
        f.write("linkage = None\n")
    for name in ("pyproj", "pycldf"):
        with open(os.path.join(stub_dir, name + ".py"), "w") as f:
            f.write("")
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, stub_dir)
    return stub_dir


def scratch_copy(rel_dir):
    """Copy an experiment directory out of the read-only tree (the reference writes results next to configs)."""
    dst = tempfile.mkdtemp(prefix="sbz_refexp_")
    target = os.path.join(dst, os.path.basename(rel_dir.rstrip("/")))
    shutil.copytree(os.path.join(REFERENCE, rel_dir), target)
    return target
