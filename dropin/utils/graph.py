"""Drop-in replacement for the reference's utils/graph.py (graph.py:10-109): preprocess_graph, make_graph
(returns the device-resident CSR graphs the HIP SpMM consumes)."""
import os
import sys

sys.path.insert(0, os.environ.get('C2DSR_AMD_ROOT', os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
from c2dsr_amd.graph import make_graph, preprocess_graph  # noqa: E402,F401
