"""HR / MRR / NDCG@{5,20} on the device (utils/metrics.py:4-31).

``RankMetrics`` accumulates the per-domain metric sums of every evaluation batch on the
device (c2dsr_rank_metrics, fp64) so an evaluation epoch needs one host sync;
``values()`` returns the reference's ``cal_metrics`` list for each domain and
``score()`` its ``cal_score`` list (improvement over a benchmark + 12 metrics).
"""
from __future__ import annotations

import torch

from . import ops


class RankMetrics:
    def __init__(self, device):
        self.sums = torch.zeros(2, 8, dtype=torch.float64, device=device)

    def add(self, rank, xory):
        ops.rank_metrics(rank, xory, 0, self.sums[0])
        ops.rank_metrics(rank, xory, 1, self.sums[1])

    def values(self):
        """([hr5, hr20, mrr5, mrr20, ndcg5, ndcg20] of domain a, same of domain b)."""
        s = self.sums.tolist()
        out = []
        for dom in (0, 1):
            if s[dom][7] > 0:
                raise IndexError('evaluation index out of range (idx_last / gt / negative item)')
            n = s[dom][6]
            if n == 0:
                raise ZeroDivisionError('no evaluation rows in this domain')  # as cal_metrics on []
            out.append([x / n for x in s[dom][:6]])
        return out[0], out[1]

    def score(self, benchmark):
        """utils/metrics.py:22-31 (cal_score): [mean improvement over benchmark] + metrics_a + metrics_b."""
        ma, mb = self.values()
        res = ma + mb
        sel = [res[0], res[4], res[6], res[10]]
        imp = [x / y - 1 for x, y in zip(sel, benchmark)]
        return [sum(imp) / len(imp)] + res
