"""Drop-in replacement for the reference's models/encoders.py (encoders.py:7-48): SelfAttention, GCN."""
import os
import sys

sys.path.insert(0, os.environ.get('C2DSR_AMD_ROOT', os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
from c2dsr_amd.models.encoders import GCN, SelfAttention  # noqa: E402,F401
