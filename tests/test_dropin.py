"""The drop-in shims (dropin/) resolve the reference's import names to this package:
main.py's `from trainer import Trainer` (main.py:8) and trainer.py's imports (trainer.py:7-9)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dropin_imports():
    code = ("import trainer, dataloader, models.C2DSR as M, models.encoders as E, utils.graph as G\n"
            "import c2dsr_amd.trainer, c2dsr_amd.models.C2DSR, c2dsr_amd.models.encoders\n"
            "assert trainer.Trainer is c2dsr_amd.trainer.Trainer\n"
            "assert M.C2DSR is c2dsr_amd.models.C2DSR.C2DSR\n"
            "assert E.SelfAttention is c2dsr_amd.models.encoders.SelfAttention and E.GCN is c2dsr_amd.models.encoders.GCN\n"
            "assert callable(dataloader.get_dataloader) and callable(G.make_graph)\n")
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, 'dropin'))
    r = subprocess.run([sys.executable, '-c', code], cwd=os.path.join(ROOT, 'dropin'), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
