"""Drop-in replacement for the reference's trainer.py (crystal22/C2DSR trainer.py:12-181).

Copy over the reference checkout's trainer.py; main.py then drives
the MI355X path unchanged via `from trainer import Trainer` (main.py:8)."""
import os
import sys

sys.path.insert(0, os.environ.get('C2DSR_AMD_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from c2dsr_amd.trainer import Trainer  # noqa: E402,F401
