"""python -m contact_zones_amd <config.json> — an sBayes experiment on the GPU
(contact_zones_amd/experiment.py; the reference's entry point is sbayes/cli.py:30-87)."""
import sys

from .experiment import main

sys.exit(main())
