"""Drop-in replacement for the reference's dataloader.py (dataloader.py:9-272): bit-exact preprocess_train /
preprocess_evaluate (same Python `random` consumption order), CDSRDataset, get_dataloader."""
import os
import sys

sys.path.insert(0, os.environ.get('C2DSR_AMD_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from c2dsr_amd.dataloader import CDSRDataset, get_dataloader  # noqa: E402,F401
