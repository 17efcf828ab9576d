"""Drop-in replacement for the reference's models/C2DSR.py (C2DSR.py:8-85): `C2DSR(args, adj, adj_specific)`
with convolve_graph / forward / forward_share and the D_a, D_b, classifier_*, embed_i* attributes."""
import os
import sys

sys.path.insert(0, os.environ.get('C2DSR_AMD_ROOT', os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
from c2dsr_amd.models.C2DSR import C2DSR  # noqa: E402,F401
