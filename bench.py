"""Training-throughput benchmark of the MI355X C2DSR path (BASELINE.json metric:
"train sequences/sec at d=256, seq_len=50, |items|~100k; 1/2/4/8 GPU").

A step = convolve_graph() + train_batch() (HIP forward, fused loss head, backward,
RCCL gradient all-reduce when N>1, fused AdamW-amsgrad) over one batch of synthetic
two-domain sequences already resident in HBM.  Workload (N=1 line): Movie-Book item
counts (36,845 + 63,937; BASELINE configs[2]), d=256, L=50, B=2048 per GPU, R=10,
dropout 0.2, at the reference's precision (fp32 results: every product on split-bf16
MFMAs with fp32 accumulation, parity 1e-4 vs the fp32 oracle).  Extra lines: the bf16
performance mode on the same workload, BASELINE configs[1] (Food-Kitchen sizes, bf16)
and configs[4] (C5 kernel roofline run).  Weak scaling: every rank trains its own batch
of B, `value` = total sequences/s over all ranks.

Launch:  python bench.py [--gpus N --steps K --warmup W]
         N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import random
import sys
import time
from types import SimpleNamespace

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n_a, n_b, d, L, B)
    'mb': dict(n_a=36845, n_b=63937, d=256, L=50, B=2048, label='Movie-Book sizes (synthetic)'),
    'fk': dict(n_a=29207, n_b=34886, d=256, L=50, B=1024, label='Food-Kitchen sizes (synthetic)'),
    'ee': dict(n_a=8367, n_b=11404, d=256, L=50, B=512, label='Entertainment-Education sizes (synthetic)'),
    'tiny': dict(n_a=2000, n_b=3000, d=64, L=20, B=256, label='tiny smoke workload'),
}
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3    # fp32-input MFMA (v_mfma_f32_32x32x2_f32, the exact-fp32 path)
# fp32 mode: each fp32-accurate product runs as three bf16 MFMAs (hi·hi + lo·hi + hi·lo, csrc/ce3.hip), so
# the matrix cores deliver at most a third of the bf16 peak in credited fp32 flops
PEAK_X3_TFLOPS = PEAK_BF16_TFLOPS / 3
PEAK_HBM_GBS = 8000.0


def log(*a):
    if int(os.environ.get('RANK', '0')) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_workload(cfg, n_seqs, seed=1):
    from c2dsr_amd import dataloader as DL
    from c2dsr_amd import graph as GR
    from c2dsr_amd import synth
    seqs = synth.make_sequences(n_seqs, cfg['n_a'], cfg['n_b'], cfg['L'], seed=seed, n_min=6)
    random.seed(3407)
    rows = DL.to_arrays(DL.preprocess_train(seqs, cfg['n_a'], cfg['n_b'], cfg['L']))
    gs, gp = GR.preprocess_graph(seqs, cfg['n_a'], cfg['n_a'] + cfg['n_b'] + 1)
    return rows, gs, gp


def make_args(cfg, device, precision, dropout=0.2, zero1=False, gnn_shard=False):
    n = cfg['n_a'] + cfg['n_b'] + 1
    return SimpleNamespace(d_latent=cfg['d'], n_item=n, n_item_a=cfg['n_a'], n_item_b=cfg['n_b'], idx_pad=n - 1,
                           shared_item_embed=False, d_bias=False, n_gnn=1, dropout_gnn=dropout, n_attn=1, n_head=1,
                           dropout_attn=dropout, norm_first=False, len_max=cfg['L'], len_rec=10, lambda_loss=0.7,
                           lr=1e-3, l2=5e-4, lr_step=10, lr_gamma=0.5, batch_size=cfg['B'], device=device,
                           precision=precision, seed=3407, zero1=zero1, gnn_shard=gnn_shard)


class KernelTimer:
    """HIP-event timing (on the stream the kernels are launched on, inside the timed region) of the
    dominant op, K5 — the fused classifier head + cross-entropy — in bf16 mode: c2dsr_ce3b_fused_fwd_u
    (online log-sum-exp AND the softmax·W part of dH in one sweep) and c2dsr_ce3b_fused_dw (ce.hip's
    c2dsr_ce_fused_* pair for other widths, the older split _fwd / _dh pair when selected).  Credited
    FLOPs: 2·M·n·d per product — forward logits, dH, dW (fwd_u carries two) — the
    logits tile the dW kernel recomputes is overhead and not credited.  fp32 mode: the split-bf16 pair
    c2dsr_ce3_fused_fwd_u / _dw."""

    NAMES_BF16 = ('c2dsr_ce3b_fused_fwd_u', 'c2dsr_ce3b_fused_dw', 'c2dsr_ce3b_fused_dw_sk', 'c2dsr_ce_fused_fwd_u',
                  'c2dsr_ce_fused_fwd', 'c2dsr_ce_fused_dh', 'c2dsr_ce_fused_dw')
    # (the dW sweep's forms, losshead.dw_plan: row splits, whole rounds + a split remainder — two launches of _dw —,
    # or stream-K, _dw_sk, whose launch includes its partial combine)
    # (round 6: with the logits kept, the forward that also stores them, _fwd_u_lg, and the dW sweeps that read them,
    # _dw_lg / _dw_lg_sk)
    NAMES_X3 = ('c2dsr_ce3_fused_fwd_u', 'c2dsr_ce3_fused_dw', 'c2dsr_ce3_fused_dw_sk', 'c2dsr_ce3_fused_fwd_u_lg',
                'c2dsr_ce3_fused_dw_lg', 'c2dsr_ce3_fused_dw_lg_sk')
    # credited products per launch: fwd_u = the lse logits + the softmax·W part of dH (online, one sweep)
    CREDIT = {'c2dsr_ce_fused_fwd_u': 2, 'c2dsr_ce3_fused_fwd_u': 2, 'c2dsr_ce3b_fused_fwd_u': 2,
              'c2dsr_ce3_fused_fwd_u_lg': 2}
    # positions of (M, n, D) in a launch's arguments (default: (Hx, Wx, bias2, M, n, D, ...))
    DIMS = {'c2dsr_ce3_fused_dw_lg': (2, 5, 6), 'c2dsr_ce3_fused_dw_lg_sk': (2, 3, 4)}

    def __init__(self, precision):
        self.names = {'bf16': self.NAMES_BF16, 'fp32': self.NAMES_X3}.get(precision, ('c2dsr_gemm',))

    def summary(self, recs):
        per = {}
        ms_all, fl_all = 0.0, 0.0
        for name in self.names:
            ms, fl = [], []
            for t, a in recs.get(name, []):
                if name == 'c2dsr_gemm':
                    f = 2.0 * a[2] * a[3] * a[4]
                    if f < 1e11:  # only the classifier-head GEMMs
                        continue
                else:  # (Hb, Wb, bias2, M, n, D, ...)
                    i, j, k = self.DIMS.get(name, (3, 4, 5))
                    f = 2.0 * a[i] * a[j] * a[k] * self.CREDIT.get(name, 1)
                ms.append(t)
                fl.append(f)
            if ms:
                per[name] = dict(launches=len(ms), avg_ms=round(sum(ms) / len(ms), 4),
                                 tflops=round(sum(fl) / (sum(ms) * 1e-3) / 1e12, 1))
                ms_all += sum(ms)
                fl_all += sum(fl)
        if not per:
            return None
        return dict(tflops=fl_all / (ms_all * 1e-3) / 1e12, ms=ms_all, per_kernel=per)


class HbmTimer:
    """HIP-event timing of the HBM-bound K1 (c2dsr_gcn_spmm) and K2 (c2dsr_embed_fwd / _bwd) launches
    inside the timed region, with ALGORITHMIC bytes per launch:

    * K1 SpMM launch over a graph of N rows and E edges, row width d (fp32):
      4·d·E (neighbour rows gathered) + 8·E (col + val) + 4·(N+1) (row pointers)
      + 4·d·N·(1 [write Y] + [Z read: self / gradient term] + [Y read: accumulate, gamma != 0] + [Y2 write])
      — fwd (n_gnn=1) = 4d(2N+E)+8E+4(N+1), bwd = 4d(3N+E)+8E+4(N+1), the survey's formulas;
    * K2 forward, per looked-up row: 16 (seq + pos int64) + 4·d·(#tables read) + 4·d (write);
      the L-row position table is cache-resident and not credited;
    * K2 backward, per row: 16 + 4·d (read dX) [+ 4·d if dXin is written]; plus 8·d per DISTINCT item
      of the batch (read-modify-write of its gradient row, ``uniq`` from the host copy of the batch).
      With dX in two compact parts (c2dsr_embed_bwd_planned_rows): per row 16 + 8 (indices, two maps), plus
      4·d per row of each part (n_q + n_k rows read), plus the 8·d per distinct item.
      Sort passes and pad-row segments are overhead, not credited."""

    NAMES = ('c2dsr_gcn_spmm', 'c2dsr_embed_fwd', 'c2dsr_embed_fwd_rows', 'c2dsr_embed_bwd', 'c2dsr_embed_bwd_planned',
             'c2dsr_embed_bwd_planned_rows', 'c2dsr_gcn_spmm_b16', 'c2dsr_embed_fwd_b16', 'c2dsr_embed_bwd_planned_b16')

    def __init__(self, n_rows_table, nnz_by_col_ptr, uniq_by_seq_ptr):
        self.N = n_rows_table
        self.nnz = nnz_by_col_ptr
        self.uniq = uniq_by_seq_ptr
        self.names = self.NAMES

    def meta_fns(self):
        """Host-side accounting evaluated at each host-side call (the C5 bf16-table backward, bench-driven): its
        first argument is the seq plan — resolved to the index tensor it sorts.  The stage operators append the
        same (and the compact parts' row count) to their own records."""
        from c2dsr_amd import ops
        return {'c2dsr_embed_bwd_planned_b16': lambda a: float(ops.PLAN_SRC.get(a[0].data_ptr(), 0))}

    def launch_bytes(self, name, a):
        """a: the call's arguments as numbers (pointers as addresses, null 0) + the meta_fns value"""
        if name in ('c2dsr_gcn_spmm', 'c2dsr_gcn_spmm_b16'):  # table bytes per element: 4, or 2 (bf16 tables)
            d, E, N, tb = int(a[7]), self.nnz[int(a[5])], self.N, (2 if name.endswith('_b16') else 4)
            from c2dsr_amd import ops
            if int(a[0]) in ops.SPMM_SLICE:  # a row slice (chunked backward, row-sharded forward): its rows and edges
                N, E = ops.SPMM_SLICE[int(a[0])]
            rows = 1 + (a[14] != 0) + (a[18] != 0.0) + (a[20] != 0)
            return tb * d * E + 8 * E + 4 * (N + 1) + tb * d * N * rows
        if name == 'c2dsr_embed_fwd':
            n, d = int(a[2]), int(a[3])
            reads = (a[4] != 0) + (a[5] != 0) + (a[6] != 0)
            return n * (16 + 4 * d * reads + 4 * d)
        if name == 'c2dsr_embed_fwd_rows':  # (seq, pos, n_rows, d, H, E, P, .., q_idx, nq, k_idx, nk, X): rows made
            k, d = int(a[13]) + int(a[15]), int(a[3])
            return k * (16 + 4 + 2 * 4 * d + 4 * d)
        n, d = int(a[2]), int(a[3])
        if name == 'c2dsr_embed_fwd_b16':  # (seq, pos, n, d, H, E, P, ..., X): two bf16 table rows, fp32 X
            return n * (16 + 2 * 2 * d + 4 * d)
        # planned backwards: the last meta value is the index tensor the seq plan sorts (its distinct items)
        if name == 'c2dsr_embed_bwd_planned_b16':  # read dX (fp32); bf16 read-modify-write per distinct item
            return n * (16 + 4 * d) + 4 * d * self.uniq.get(int(a[-1]), 0)
        if name == 'c2dsr_embed_bwd_planned_rows':  # (.., n, d, gXa, inv_a, gXb, inv_b, ..) + (rows of parts, seq)
            return n * (16 + 8) + 4 * d * a[-2] + 8 * d * self.uniq.get(int(a[-1]), 0)
        if name == 'c2dsr_embed_bwd_planned':  # (seq_plan, pos_plan, n, d, gX, .., G, n_items, gP, n_pos, gXin, ..)
            return n * (16 + 4 * d + (4 * d if a[14] != 0 else 0)) + 8 * d * self.uniq.get(int(a[-1]), 0)
        return n * (16 + 4 * d + (4 * d if a[14] != 0 else 0)) + 8 * d * self.uniq.get(int(a[0]), 0)

    def summary(self, recs, steps):
        per, tb, tms = {}, 0.0, 0.0
        for name in self.NAMES:
            rec = recs.get(name, [])
            if not rec:
                continue
            ms = sum(t for t, _ in rec)
            by = sum(self.launch_bytes(name, a) for _, a in rec)
            per[name] = dict(launches=len(rec), avg_ms=round(ms / len(rec), 4), gbs=round(by / (ms * 1e-3) / 1e9, 1),
                             bytes_per_launch=int(by / len(rec)))
            tb += by
            tms += ms
        if not per:
            return None
        ach = tb / (tms * 1e-3) / 1e9
        # north_star names "embedding-gather + GNN-SpMM": the same accounting over those kernels alone (the forward
        # gathers and both SpMM directions), next to the whole K1 + K2 figure that also carries the backward's
        # deterministic segment sums
        gs = [n for n in per if 'spmm' in n or 'embed_fwd' in n]
        gb = sum(per[n]['bytes_per_launch'] * per[n]['launches'] for n in gs)
        gms = sum(per[n]['avg_ms'] * per[n]['launches'] for n in gs)
        gather_spmm = None
        if gms > 0:
            ga = gb / (gms * 1e-3) / 1e9
            gather_spmm = dict(achieved=round(ga, 1), frac=round(ga / PEAK_HBM_GBS, 4), kernels=gs)
        return dict(bound='hbm', achieved=round(ach, 1), peak=PEAK_HBM_GBS, unit='GB/s', frac=round(ach / PEAK_HBM_GBS, 4),
                    traffic=None, kernel='K1 c2dsr_gcn_spmm (fwd+bwd) + K2 c2dsr_embed_fwd/bwd; algorithmic bytes '
                    '(bench.py HbmTimer)', ms_per_step=round(tms / steps, 4), per_kernel=per,
                    gather_spmm=gather_spmm)


def timing_begin(*timers):
    """Bracket the timers' entry points with HIP events from here on (c2dsr::timing_set)."""
    from c2dsr_amd._lib import lib
    lib.time_meta = {}
    for t in timers:
        if hasattr(t, 'meta_fns'):
            lib.time_meta.update(t.meta_fns())
    lib.timing_start(sorted({n for t in timers for n in t.names}))


def timing_end():
    """Stop timing; the records of every bracketed call since timing_begin (name -> [(ms, args)])."""
    from c2dsr_amd._lib import lib
    torch.cuda.synchronize()
    recs = lib.timing_take()
    lib.timing_start([])
    lib.time_meta = {}
    return recs


def uniq_counts(batches, host):
    """data_ptr of every device index tensor of the batches -> number of distinct items in it (counted on the
    host copies: no device sort in the profiled process)."""
    out = {}
    for b, h in zip(batches, host):
        for j in (0, 1, 2, 12, 13):  # seq_share, seq_a, seq_b, neg_a, neg_b
            out[b[j].data_ptr()] = int(np.unique(h[j]).size)
    return out


def k5_traffic(precision):
    """HBM bytes per K5 launch set of one head (fwd_u + rows + dW kernels, both heads averaged) from the separate
    rocprofv3 FETCH_SIZE (x2, the gfx950 correction) / WRITE_SIZE passes of tools/round_profile.sh,
    summarised by tools/pmc_traffic.py into profiles/k5_traffic.json.  PMC counters cannot be read
    from inside this process, so the committed measurement of the same code is reported (null if
    absent or for another precision)."""
    path = os.path.join(ROOT, 'profiles', {'bf16': 'k5_traffic.json', 'fp32': 'k5_traffic_fp32.json'}.get(precision, '-'))
    if not os.path.exists(path):
        return None, None, None
    with open(path) as f:
        t = json.load(f)
    return t.get('bytes_per_head', t.get('bytes_per_launch_triple')), t.get('source'), t.get('mfma_busy')


def hbm_traffic(precision):
    """K1 + K2 HBM bytes per step (all their launches) from the same PMC passes (profiles/hbm_traffic.json,
    tools/pmc_traffic.py): measured DRAM traffic below the algorithmic bytes means the MALL / L2 served
    part of the gathers (re-read table rows)."""
    path = os.path.join(ROOT, 'profiles', 'hbm_traffic.json' if precision == 'bf16' else 'hbm_traffic_fp32.json')
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    return t.get('bytes_per_step'), t.get('source')


# the GPU kernels behind each timed C-ABI entry point (PMC counters are per GPU kernel; the embedding backward's
# segment sums are the ROLE 0 instantiations — tools/pmc_traffic.py)
SEG0 = ('seg_chunk_kernel<64, 0>', 'seg_split1_kernel<64, 0>', 'seg_split2_kernel<64, 0>')
DRAM_KERNELS = {'c2dsr_gcn_spmm': ('spmm_kernel', 'spmm_pf_kernel', 'spmm_nc_kernel', 'combine_kernel'),
                'c2dsr_gcn_spmm_b16': ('spmm_kernel', 'spmm_pf_kernel', 'combine_kernel'),
                'c2dsr_embed_fwd': ('embed_fwd_kernel',), 'c2dsr_embed_fwd_b16': ('embed_fwd_kernel',),
                'c2dsr_embed_fwd_rows': ('embed_fwd_rows_kernel',),
                'c2dsr_embed_bwd_planned': SEG0, 'c2dsr_embed_bwd_planned_rows': SEG0, 'c2dsr_embed_bwd_planned_b16': SEG0}


def add_dram(roof, path, steps):
    """DRAM-side fractions beside the algorithmic ones: the PMC bytes per step of the same
    kernels (profiles/*traffic*.json: rocprofv3 FETCH_SIZE ×2 + WRITE_SIZE passes, tools/pmc_traffic.py) over the
    kernels' time measured here.  Algorithmic bytes credit every gathered row, so a Zipf-popular row served from
    L2 / MALL counts each time it is read; the DRAM figure counts what left HBM.  An entry point whose kernels the
    PMC file does not cover gets no DRAM figure."""
    if roof is None or not os.path.exists(path):
        return
    with open(path) as f:
        t = json.load(f)
    pk = t.get('per_kernel', {})
    tot_b, tot_ms = 0.0, 0.0
    for name, rec in roof['per_kernel'].items():
        ks = [k for k in DRAM_KERNELS.get(name, ()) if k in pk]
        if not ks:
            continue
        by = sum(pk[k]['bytes'] for k in ks)  # per step
        ms = rec['avg_ms'] * rec['launches'] / steps
        rec['dram_gbs'] = round(by / (ms * 1e-3) / 1e9, 1)
        rec['dram_frac'] = round(rec['dram_gbs'] / PEAK_HBM_GBS, 4)
        tot_b += by
        tot_ms += ms
    gs = roof.get('gather_spmm')
    if gs:
        recs = [roof['per_kernel'][n] for n in gs['kernels'] if 'dram_gbs' in roof['per_kernel'][n]]
        if recs:
            b = sum(r['dram_gbs'] * r['avg_ms'] * r['launches'] for r in recs)
            gs['dram_achieved'] = round(b / sum(r['avg_ms'] * r['launches'] for r in recs), 1)
            gs['dram_frac'] = round(gs['dram_achieved'] / PEAK_HBM_GBS, 4)
    if tot_ms > 0:
        roof['dram_achieved'] = round(tot_b / (tot_ms * 1e-3) / 1e9, 1)
        roof['dram_frac'] = round(roof['dram_achieved'] / PEAK_HBM_GBS, 4)
        roof['dram_source'] = (f'{t.get("source")} ({os.path.basename(path)}): PMC DRAM bytes per step / kernel '
                               'time here; achieved / frac stay algorithmic (SURVEY §8(d))')


def flag_above_peak(roof):
    """A per-kernel algorithmic rate above the HBM peak is L2 / MALL hits on re-read (Zipf-popular) rows, not a
    faster memory: such an entry always carries its DRAM-side figure, or says it has none."""
    if not roof:
        return
    for rec in roof.get('per_kernel', {}).values():
        if rec.get('gbs', 0) > PEAK_HBM_GBS and 'dram_gbs' not in rec:
            rec['above_peak_note'] = ('algorithmic bytes count every gathered row; rows re-read from L2 / MALL make '
                                      'this exceed the HBM peak — no PMC DRAM figure for this kernel in this run')


def cpu_threads():
    """The host threads the CPU baseline uses: the box's CPU share for one GPU (OMP_NUM_THREADS, 16 on the
    GPU box; os.cpu_count() there reports the whole machine, whose other cores belong to other jobs)."""
    share = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or 16
    return max(1, min(os.cpu_count() or 1, share))


def cpu_baseline(cfg, rows, gs, gp, budget_s=20.0, min_steps=1):
    """The oracle (CPU fp32 restatement, oracle/c2dsr_oracle.py) on a bounded sample of the same
    workload at the configuration's own batch: same item tables, d, L,
    B; one untimed warm-up step, then timed steps until ``budget_s`` is spent and at least ``min_steps``."""
    sys.path.insert(0, ROOT)
    from oracle import c2dsr_oracle as O
    from c2dsr_amd.models.C2DSR import C2DSR
    threads = cpu_threads()
    torch.set_num_threads(threads)
    args = make_args(cfg, torch.device('cpu'), 'fp32')
    torch.manual_seed(0)
    model = C2DSR(args, gs, gp)
    params = {n: p.detach().clone() for n, p in model.named_parameters()}
    del model
    graphs = {}
    for k, g in (('share', gs), ('specific', gp)):
        r, c, v = g.coo()
        graphs[k] = (torch.from_numpy(r), torch.from_numpy(c), torch.from_numpy(v))
    ocfg = O.cfg_from_args(args)
    tr = O.OracleTrainer(params, graphs, ocfg, seed=3407)
    Bs = cfg['B']
    n_rows = rows[0].shape[0]
    steps, done, el = 0, 0, 0.0
    while True:
        lo = (steps * Bs) % max(1, n_rows - Bs)
        b = tuple(torch.from_numpy(r[lo:lo + Bs].copy()) for r in rows)
        t0 = time.time()
        tr.train_batch(b)
        if steps > 0:  # the first step is the warm-up
            el += time.time() - t0
            done += Bs
            log(f'[bench] cpu baseline step {steps}: {time.time() - t0:.1f}s')
            if el > budget_s and done // Bs >= min_steps:
                break
        steps += 1
    return dict(value=round(done / el, 3), unit='train sequences/sec', cores=threads, kind='port',
                sample=f'oracle (torch-CPU fp32 restatement) train step, {cfg["label"]}, d={cfg["d"]}, '
                       f'L={cfg["L"]}, batch {Bs}, 1 warm-up + {done // Bs} timed steps '
                       f'(budget {budget_s:.0f} s, at least {min_steps}), dropout 0.2, {threads} host threads '
                       '(the box\'s CPU share for one GPU)')


def run_c5(opt, world, rank, device, emit=True):
    """BASELINE configs[4] / SURVEY.md §8(d) C5 as a kernel roofline run: synthetic two-domain
    10M + 10M items, d=512, L=100, B=8192 global (8192/N per GPU, weak per-GPU work at N=8: 1024),
    graph from 2M sequences.  A full replicated model is infeasible (164 GB of fp32 parameters before
    optimizer state, ~13 TB of logits), so a step is the HBM-bound part of the training step on the
    shared table: K1 GCN forward (A·drop(E), mean) + the five K2 embedding gathers (share, a, b, neg_a,
    neg_b index sets) forward + their deterministic backward + the K1 GCN backward through Aᵀ into
    E.grad.  The line's value is on bf16 [N, d] tables (E, H, the lookup gradient and E.grad,
    4 × 20.5 GB; the *_b16 kernels, fp32 arithmetic); ``fp32_tables`` is the same step on fp32 tables through the
    product's autograd functions (ops.GCNFn / ops.EmbedFn).  Value = algorithmic GB/s of those kernels
    (HbmTimer); each rank works on its own batch (no exchange)."""
    from c2dsr_amd import dataloader as DL
    from c2dsr_amd import graph as GR
    from c2dsr_amd import ops, synth
    from c2dsr_amd import dropout as DK
    from c2dsr_amd.models.encoders import GCN, StepState
    n_a = n_b = 10_000_000
    d, L = 512, 100
    N = n_a + n_b + 1
    B = opt.batch or 1024  # 8192 global over the 8 GPUs of the node
    t0 = time.time()
    items, off = synth.make_flat_sequences(opt.c5_seqs, n_a, n_b, L, seed=1)
    seq_id = np.repeat(np.arange(off.size - 1, dtype=np.int64), np.diff(off))
    same = seq_id[1:] == seq_id[:-1]
    share = np.stack([items[:-1][same], items[1:][same]], 1)
    del seq_id, same
    g = GR.normalized_csr(share, N)
    del share
    log(f'[c5] {off.size - 1} sequences, {items.size} interactions, share graph nnz {g.nnz}, '
        f'prep {time.time() - t0:.1f}s')
    first = rank * B  # this rank's batch rows
    seqs = [items[off[i]:off[i + 1]].tolist() for i in range(first * 2, first * 2 + 2 * B)]
    random.seed(3407)
    rows = DL.to_arrays(DL.preprocess_train(seqs, n_a, n_b, L))  # drops sequences without targets
    assert rows[0].shape[0] >= B, rows[0].shape
    del items, off
    dg = GR.DeviceGraph(g, device)
    b = [torch.from_numpy(r[:B].copy()).to(device) for r in rows]
    passes = [(b[0], b[3]), (b[1], b[4]), (b[2], b[5]), (b[12], b[3]), (b[13], b[3])]
    nnz = {}
    for t in (False, True):
        col = dg.plan(t)[5]
        nnz[col.data_ptr()] = col.numel()
    uniq = {seq.data_ptr(): int(np.unique(rows[j][:B]).size) for j, (seq, _) in zip((0, 1, 2, 12, 13), passes)}
    p = 0.2

    def measure(b16):
        torch.manual_seed(0)
        gx = torch.empty(B, L, d, device=device).normal_(0.0, 1e-3)
        args = SimpleNamespace(dropout_gnn=p, n_gnn=1, idx_pad=N - 1)
        state = StepState(seed=3407)
        gcn = GCN(args)
        gcn.state = state
        if b16:  # E, H, the lookup gradient G and E.grad as bf16 [N, d] tables (4 × 20.5 GB), fp32 arithmetic
            from c2dsr_amd._lib import lib, stream
            E = torch.empty(N, d, device=device, dtype=torch.bfloat16).normal_(0.0, 0.1)
            H, G, gE = torch.empty_like(E), torch.empty_like(E), torch.zeros_like(E)
            P = torch.empty(L, d, device=device).normal_(0.0, 0.1)
            gP = torch.zeros_like(P)
            x = torch.empty(B, L, d, device=device)
            ws_bytes = int(lib.raw('c2dsr_embed_bwd_planned_workspace')(B * L, d))
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
        else:
            E = torch.nn.Parameter(torch.empty(N, d, device=device).normal_(0.0, 0.1))
            E.grad = torch.zeros_like(E)
            P = torch.nn.Parameter(torch.empty(L, d, device=device).normal_(0.0, 0.1))
            P.grad = torch.zeros_like(P)

        def step_fp32():  # the product's autograd functions (ops.GCNFn / ops.EmbedFn)
            state.step += 1
            H, tok, sink = gcn.propagate(E, dg)
            xs = []
            for k, (seq, pos) in enumerate(passes):
                keys = state.keys(DK.site_enc(k, 0, DK.K_INPUT))
                xs.append(ops.EmbedFn.apply(tok, E, P, seq, pos, H, math.sqrt(d), p, keys, rank * B, sink, N - 1))
            torch.autograd.backward(xs, [gx] * len(xs))

        def step_b16():
            # the same kernels on bf16 tables (the fused GCN / embedding autograd functions' launches, by hand):
            # H = (E + A·drop(E))/2; five gathers; G = Σ segment sums of the five passes; E.grad += (drop(AᵀG) +
            # G)/2 + [i != pad]·G (ops.GCNFn.backward with n_gnn = 1)
            state.step += 1
            pg, gkeys = gcn._keys()
            ops.spmm(dg, False, E, gkeys[0], pg, 0, 0.5, E, 0.5, 0.0, -1, 0.0, H)
            plans = ops.index_plans(state, [(seq, N) for seq, _ in passes] + [(pos, L) for _, pos in passes])
            ekeys = [state.keys(DK.site_enc(k, 0, DK.K_INPUT)) for k in range(len(passes))]
            for k, (seq, pos) in enumerate(passes):  # forward (x is consumed by nothing else here)
                lib('c2dsr_embed_fwd_b16', seq, pos, B * L, d, H, E, P, math.sqrt(d), ekeys[k][0], ekeys[k][1], p,
                    rank * B * L, x, N, L, None, stream())
            G.zero_()
            for k, (seq, pos) in enumerate(passes):
                lib('c2dsr_embed_bwd_planned_b16', plans[k].get(), plans[len(passes) + k].get(), B * L, d, gx,
                    ekeys[k][0], ekeys[k][1], p, rank * B * L, math.sqrt(d), G, N, gP, L, ws, ws_bytes, stream())
            ops.spmm(dg, True, G, gkeys[0], pg, 1, 0.5, G, 0.5, 1.0, N - 1, 1.0, gE)

        step = step_b16 if b16 else step_fp32
        ht = HbmTimer(N, nnz, uniq)
        for _ in range(opt.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        timing_begin(ht)
        t0 = time.perf_counter()
        for _ in range(opt.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        recs = timing_end()
        if world > 1:
            t = torch.tensor([el], device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        return ht.summary(recs, opt.steps), el

    modes = ['bf16', 'fp32'] if opt.c5_tables == 'both' else [opt.c5_tables]
    res = {}
    for m in modes:
        res[m] = measure(m == 'bf16')
        torch.cuda.empty_cache()
    roof, el = res[modes[0]]
    out = None
    if rank == 0:
        out = {'metric': 'C5 HBM roofline: K1 GCN SpMM + K2 embedding gather (fwd+bwd), algorithmic GB/s',
               'value': round(roof['achieved'] * world, 1), 'unit': 'GB/s (all ranks)', 'n_gpus': world,
               'steps': opt.steps, 'warmup': opt.warmup, 'ms_per_step': round(el / opt.steps * 1e3, 3),
               'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
               'data': 'synthetic (Zipf two-domain sequences, vectorised generator)',
               'config': {'workload': 'c5: synthetic 10M+10M items, d=512, L=100 (BASELINE configs[4])',
                          'tables': modes[0],
                          'n_item': N, 'd': d, 'seq_len': L, 'batch_per_gpu': B, 'global_batch': B * world,
                          'graph_sequences': opt.c5_seqs, 'graph_nnz': g.nnz, 'dropout': p,
                          'parallelism': f'dp{world}'},
               'roofline': roof, 'cpu_baseline': None}
        tpath = os.path.join(ROOT, 'profiles', 'c5_traffic.json')
        if modes[0] == 'bf16' and os.path.exists(tpath):  # PMC DRAM bytes of the same step (tools/pmc_traffic.py c5)
            with open(tpath) as f:
                t = json.load(f)
            roof['traffic'] = t.get('bytes_per_step')
            roof['traffic_unit'] = 'bytes per step (all K1+K2 launches); achieved/peak use algorithmic bytes'
            roof['traffic_source'] = t.get('source')
            add_dram(roof, tpath, opt.steps)
        flag_above_peak(roof)
        for m in modes[1:]:  # the other table storage on the same graph and batch
            r2, el2 = res[m]
            tpath2 = os.path.join(ROOT, 'profiles', f'c5_traffic_{m}.json')  # its own PMC passes (--c5-tables fp32)
            if os.path.exists(tpath2):
                with open(tpath2) as f:
                    t2 = json.load(f)
                r2['traffic'] = t2.get('bytes_per_step')
                r2['traffic_unit'] = 'bytes per step (all K1+K2 launches); achieved/peak use algorithmic bytes'
                r2['traffic_source'] = t2.get('source')
                add_dram(r2, tpath2, opt.steps)
            flag_above_peak(r2)
            out[f'{m}_tables'] = {'value': round(r2['achieved'] * world, 1),
                                  'ms_per_step': round(el2 / opt.steps * 1e3, 3), 'roofline': r2}
        if emit:
            print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='mb', choices=list(CONFIGS) + ['c5'])
    ap.add_argument('--precision', default='fp32', choices=['bf16', 'fp32', 'fp32_exact'])
    ap.add_argument('--batch', type=int, default=0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-budget', type=float, default=20.0)
    ap.add_argument('--c5-seqs', type=int, default=2_000_000)
    ap.add_argument('--c5-tables', default='both', choices=['bf16', 'fp32', 'both'],
                    help='C5 [N, d] table storage (SURVEY.md §8(d): bf16 tables, the line\'s value; fp32 = the '
                         'product\'s autograd path; both: bf16 line + fp32_tables sub-object on the same graph)')
    ap.add_argument('--no-extra', dest='extra', action='store_false',
                    help='skip the extra lines (MB bf16 mode, FK bf16, C5) of the default N=1 run')
    ap.add_argument('--no-c5', dest='c5_extra', action='store_false', help='skip the C5 extra line')
    ap.add_argument('--no-c4', dest='c4_extra', action='store_false', help='skip the C4 strong-scaling model line')
    ap.add_argument('--zero1', action='store_true',
                    help='N>1: ZeRO-1 (reduce-scatter, 1/p AdamW, all-gather; c2dsr_amd/dp.py) for the main line')
    ap.add_argument('--gnn-shard', action='store_true',
                    help='N>1: row-sharded GCN propagation (each rank propagates N/p rows, all-gather; ops.RowShard) '
                         'for the main line')
    ap.add_argument('--dp-split', action='store_true',
                    help='strong scaling: every rank trains its slice of the same global batch (BASELINE '
                         'configs[3], e.g. --config ee --batch 4096)')
    opt = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    device = torch.device('cuda', 0)
    if world > 1:
        # the trainer's own set-up (c2dsr_amd.trainer.init_data_parallel): the rank's device is cuda:LOCAL_RANK (modulo
        # the visible devices), the group RCCL when every rank drives its own GPU (device identities exchanged over
        # the launcher's store), gloo only when ranks share one (a rehearsal on a smaller box); C2DSR_DP_BACKEND
        # (or the older C2DSR_DIST_BACKEND) overrides
        from types import SimpleNamespace
        from c2dsr_amd.trainer import init_data_parallel
        if os.environ.get('C2DSR_DIST_BACKEND') and not os.environ.get('C2DSR_DP_BACKEND'):
            os.environ['C2DSR_DP_BACKEND'] = os.environ['C2DSR_DIST_BACKEND']
        ns = SimpleNamespace(device=torch.device('cuda', 0))
        rank, world = init_data_parallel(ns)
        device = ns.device
        log(f'[bench] rank {rank}/{world} on {device} ({dist.get_backend()})')
    if opt.config == 'c5':
        run_c5(opt, world, rank, device)
        if world > 1:
            dist.destroy_process_group()
        return
    cfg = dict(CONFIGS[opt.config])
    if opt.batch:
        cfg['B'] = opt.batch
    wl = workload(cfg, opt.config)
    res = run_train(opt, cfg, opt.config, opt.precision, wl, world, rank, device)
    extra = {}
    if world > 1 and opt.extra:
        # the other exchange of the N>1 path: ZeRO-1 if the main line replicated AdamW,
        # else the replicated all-reduce — same workload, same ranks
        torch.cuda.empty_cache()
        alt = not opt.zero1
        r2 = run_train(opt, cfg, opt.config, opt.precision, wl, world, rank, device, zero1=alt)
        if rank == 0:
            extra['dp_zero1' if alt else 'dp_allreduce'] = brief(r2)
        # the other GCN propagation of the N>1 path: row-sharded + all-gather, or replicated
        torch.cuda.empty_cache()
        r4 = run_train(opt, cfg, opt.config, opt.precision, wl, world, rank, device, gnn_shard=not opt.gnn_shard)
        if rank == 0:
            extra['dp_gnn_replicated' if opt.gnn_shard else 'dp_gnn_shard'] = brief(r4)
        if opt.config == 'mb' and not opt.batch:
            # BASELINE configs[3] (C4): Entertainment-Education sizes, B=4096 global split over the ranks
            # (strong scaling), the same exchange as the main line
            torch.cuda.empty_cache()
            ee = dict(CONFIGS['ee'], B=4096)
            r3 = run_train(opt, ee, 'ee', opt.precision, workload(ee, 'ee'), world, rank, device, dp_split=True)
            if rank == 0:
                extra['ee_c4_split'] = brief(r3)
    if rank == 0:
        if world == 1 and opt.extra and opt.config == 'mb' and not opt.batch:
            # driver-visible lines of the other single-GPU configurations: the other precision mode on the same
            # workload, and BASELINE configs[1] (Food-Kitchen sizes, B=1024, bf16 as BASELINE names it)
            other = 'bf16' if opt.precision != 'bf16' else 'fp32'
            extra[f'mb_{other}'] = brief(run_train(opt, cfg, 'mb', other, wl, world, rank, device))
            torch.cuda.empty_cache()
            fk = dict(CONFIGS['fk'])
            wfk = workload(fk, 'fk')
            extra['fk_bf16'] = brief(run_train(opt, fk, 'fk', 'bf16', wfk, world, rank, device))
            del wfk
            torch.cuda.empty_cache()
            if opt.c4_extra:  # BASELINE configs[3]: the strong-scaling model of C4 from two one-GPU points
                extra['c4_strong'] = c4_strong(opt, rank, device)
                torch.cuda.empty_cache()
            if opt.c5_extra:  # BASELINE configs[4]: the K1 + K2 HBM roofline run at 10M + 10M items, d = 512
                extra['c5_hbm'] = run_c5(opt, world, rank, device, emit=False)
                torch.cuda.empty_cache()
        cpu = None
        if world == 1 and not opt.no_cpu_baseline:
            cpu = cpu_baseline(cfg, *wl, opt.cpu_budget)
            if opt.config == 'mb' and opt.extra:
                # the same restatement at configs[0] (C1: Food-Kitchen item counts, d=64, L=15,
                # B=128 — the reference's own CPU-runnable case) for at least five timed steps
                c1 = dict(n_a=29207, n_b=34886, d=64, L=15, B=128, label='Food-Kitchen sizes (synthetic), C1')
                cpu['extra'] = {'c1_fk_d64': cpu_baseline(c1, *workload(c1, 'c1'), budget_s=5.0, min_steps=5)}
                # and at configs[1] (C2: Food-Kitchen sizes, d=256, L=50, B=1024; one timed step ≈ 20 s)
                fk = dict(CONFIGS['fk'])
                cpu['extra']['c2_fk_d256'] = cpu_baseline(fk, *workload(fk, 'fk'), budget_s=10.0, min_steps=1)
        res['cpu_baseline'] = cpu
        if extra:
            res['extra_lines'] = extra
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


XGMI_BUSBW_GBS = (300.0, 600.0)  # assumed RCCL all-reduce bus bandwidth on 8 × MI355X (conservative, optimistic)


def c4_strong(opt, rank, device):
    """BASELINE configs[3] (C4: Entertainment-Education sizes, B = 4096 global over 8 GPUs, strong scaling) modelled
    from two one-GPU runs (T(p) = F + V/p, target ≥ 6× at p = 8):
      T(4096) = F + V and T(512) = F + V/8  ⇒  V = 8/7·(T(4096) − T(512)),  F = T(4096) − V,
    F = the per-step work that does not shrink with the per-GPU batch (GCN propagation fwd + bwd over the whole item
    graph, AdamW over all parameters, launch overheads), V = the batch-proportional part.  At p = 8 each rank also
    all-reduces the flat fp32 gradient (4·n_params bytes; ring: 2·7/8 of it per GPU) — issued range by range inside
    the backward (c2dsr_amd/dp.py), so only the last table chunk is exposed; the projection charges the WHOLE
    all-reduce as exposed (upper bound on T(8)) and, separately, the last chunk only."""
    ee = CONFIGS['ee']
    pts = {}
    for B in (4096, 512):
        c = dict(ee, B=B)
        wl = workload(c, 'ee')
        pts[B] = run_train(opt, c, 'ee', opt.precision, wl, 1, rank, device)
        del wl
        torch.cuda.empty_cache()
    t8, t1 = pts[512]['ms_per_step'], pts[4096]['ms_per_step']
    V = 8.0 / 7.0 * (t1 - t8)
    F = t1 - V
    n_params = pts[4096]['n_params']
    wire = 2 * 7 / 8 * 4 * n_params  # bytes per GPU of a ring all-reduce over 8 ranks
    n_item = ee['n_a'] + ee['n_b'] + 1
    last_chunk = 4 * n_item * ee['d'] / 4  # one of the 4 row chunks of the last item table (dp.TABLE_CHUNKS)
    proj = {}
    for bw in XGMI_BUSBW_GBS:
        ar = wire / (bw * 1e9) * 1e3
        ex = 2 * 7 / 8 * last_chunk / (bw * 1e9) * 1e3
        proj[f'busbw_{int(bw)}GBs'] = dict(allreduce_ms=round(ar, 3), exposed_tail_ms=round(ex, 4),
                                           T8_ms_all_exposed=round(F + V / 8 + ar, 3),
                                           speedup_all_exposed=round(t1 / (F + V / 8 + ar), 2),
                                           T8_ms_tail_exposed=round(F + V / 8 + ex, 3),
                                           speedup_tail_exposed=round(t1 / (F + V / 8 + ex), 2))
    return dict(b4096=brief(pts[4096]), b512=brief(pts[512]), F_ms=round(F, 3), V_ms=round(V, 3),
                F_over_V=round(F / V, 4) if V > 0 else None, n_params=n_params, grad_bytes=4 * n_params,
                projection_p8=proj, ideal_speedup_p8=round(t1 / (F + V / 8), 2),
                note='one-GPU measurements; T(p) = F + V/p (SURVEY §8(e)); all-reduce at an assumed xGMI bus '
                     'bandwidth (no 8-GPU node here)')


def workload(cfg, name):
    """The synthetic workload of a configuration, pinned: 20·B sequences (≥ 20·B_global)
    from the fixed generator seed, and the graphs built from them — independent of --steps / --warmup."""
    t_prep = time.time()
    rows, gs, gp = make_workload(cfg, 20 * cfg['B'] if name != 'tiny' else 4 * cfg['B'], seed=1)
    log(f'[bench] {cfg["label"]}: {rows[0].shape[0]} train sequences, graph nnz {gs.nnz}/{gp.nnz}, '
        f'prep {time.time() - t_prep:.1f}s')
    return rows, gs, gp


def brief(r):
    keep = ('value', 'unit', 'ms_per_step', 'dtype', 'config', 'loss', 'n_gpus', 'host_prep')
    out = {k: r[k] for k in keep}
    for k in ('roofline', 'roofline_hbm'):
        if r.get(k):
            out[k] = {kk: r[k][kk] for kk in ('bound', 'achieved', 'peak', 'unit', 'frac', 'ms_per_step', 'gather_spmm',
                                              'dram_achieved', 'dram_frac') if kk in r[k]}
    return out


def run_train(opt, cfg, name, precision, wl, world, rank, device, zero1=None, dp_split=None, gnn_shard=None):
    """W untimed + K timed training steps of one configuration; returns the bench line (rank 0)."""
    rows, gs, gp = wl
    B = cfg['B']
    n_rows = rows[0].shape[0]
    n_batches = opt.steps + opt.warmup
    from c2dsr_amd.trainer import Trainer
    zero1 = opt.zero1 if zero1 is None else zero1
    dp_split = opt.dp_split if dp_split is None else dp_split
    gnn_shard = opt.gnn_shard if gnn_shard is None else gnn_shard
    args = make_args(cfg, device, precision, zero1=zero1 and world > 1, gnn_shard=gnn_shard and world > 1)
    torch.manual_seed(3407)
    tr = Trainer(args, None, data=(None, None, None), graphs=(gs, gp))
    tr.dp_split = dp_split
    B_local = B if not dp_split else -(-B // world)
    batches, host = [], []
    for i in range(n_batches):
        # weak scaling: rank r trains batch (i·world + r); dp_split: all ranks slice the same global batch
        j = i * world + rank if not dp_split else i
        lo = (j * B) % max(1, n_rows - B)
        host.append(tuple(r[lo:lo + B] for r in rows))
        batches.append(tuple(torch.from_numpy(r[lo:lo + B].copy()).to(device) for r in rows))
    timer = KernelTimer(precision)
    dgs = tr.model.graphs()
    nnz = {}
    for g in dgs:
        for t in (False, True):
            col = g.plan(t)[5]
            nnz[col.data_ptr()] = col.numel()
    htimer = HbmTimer(tr.model.n_item, nnz, uniq_counts(batches, host))
    tr.model.train()
    tr.optimizer.zero_grad()
    B_global = B * world if not dp_split else B

    # the launch sizes of every step (compact row sets, padding rows, valid targets), counted by the data pipeline
    # from the batches' host arrays as it stages them — so no count is read back from the device inside a step
    t_cnt = time.perf_counter()
    counts = [tr.launch_counts(h, global_rows=B_global) for h in host]
    host_counts_ms = (time.perf_counter() - t_cnt) * 1e3 / max(1, len(host))

    def step(i):
        tr.model.convolve_graph()
        return tr.train_batch(batches[i], global_rows=B_global, counts=counts[i])

    for i in range(opt.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timing_begin(timer, htimer)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for i in range(opt.steps):
        last = step(opt.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    recs = timing_end()
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    loss = float(last[0].detach())
    ks = timer.summary(recs)
    hb = htimer.summary(recs, opt.steps)
    ms = el / opt.steps * 1e3
    value = B_global * opt.steps / el
    n_params = int(tr.model.flat.numel)
    del tr, batches
    peak = {'bf16': PEAK_BF16_TFLOPS, 'fp32': PEAK_X3_TFLOPS}.get(precision, PEAK_FP32_TFLOPS)
    roof = None
    if ks is not None:
        traffic, tsrc, busy = k5_traffic(precision) if name == 'mb' else (None, None, None)
        roof = dict(bound='mfma', achieved=round(ks['tflops'], 2), peak=peak, unit='TFLOP/s',
                    frac=round(ks['tflops'] / peak, 4), traffic=traffic, traffic_source=tsrc,
                    kernel={'bf16': 'K5 fused classifier head + CE: ce3_kernel<256,0,bf16> (lse + dH, online) + '
                                    'ce3_kernel<256,1,bf16> (dW), one bf16 MFMA per product; credited 2·Mv·n·d per '
                                    'product over the Mv valid rows (fwd_u 2, dw 1)',
                            'fp32': 'K5 fused classifier head + CE at fp32 accuracy: ce3_kernel<256,0> (lse + dH, '
                                    'online; with the logits kept it also stores them) + the dW sweep — '
                                    'ce3_dwl_kernel on the stored logits (losshead.CE_LOGITS, the default) or '
                                    'ce3_kernel<256,1> recomputing them —, split-bf16 operands, 3 bf16 MFMAs per '
                                    'product; credited 2·Mv·n·d per fp32 product over the Mv valid rows (fwd_u 2, '
                                    'dw 1); peak = bf16 dense peak / 3'}.get(
                        precision, 'gemm_kernel (K5 materialised logits GEMMs, fp32-input MFMA)'),
                    ms_per_step=round(ks['ms'] / opt.steps, 4), per_kernel=ks['per_kernel'],
                    mfma_busy=busy, mfma_busy_note='SQ_VALU_MFMA_BUSY_CYCLES / SIMD cycles of the K5 launches '
                    '(same PMC run as traffic; counts any recomputed logits tiles, which frac does not credit)')
    if hb is not None and name == 'mb' and precision in ('bf16', 'fp32'):
        hb['traffic'], hb['traffic_source'] = hbm_traffic(precision)
        hb['traffic_unit'] = 'bytes per step (all K1+K2 launches); achieved/peak use algorithmic bytes'
        add_dram(hb, os.path.join(ROOT, 'profiles', 'hbm_traffic.json' if precision == 'bf16'
                                  else 'hbm_traffic_fp32.json'), opt.steps)
    flag_above_peak(hb)
    par = (f'dp{world}' + ('-split' if dp_split and world > 1 else '') + ('-zero1' if zero1 and world > 1 else '')
           + ('-gnnshard' if gnn_shard and world > 1 else ''))
    return {'metric': 'train sequences/sec at d=256, seq_len=50, |items|~100k',
            'value': round(value, 2), 'unit': 'train sequences/sec', 'n_gpus': world, 'steps': opt.steps,
            'warmup': opt.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True,
            'scaling': 'strong' if dp_split and world > 1 else 'weak',
            'vs_baseline': None, 'dtype': {'fp32': 'f32', 'bf16': 'bf16', 'fp32_exact': 'f32'}[precision],
            'precision_mode': {'fp32': 'fp32 results, split-bf16 x3 MFMA products (reference parity 1e-4)',
                               'bf16': 'bf16 MFMA operands, fp32 accumulate and storage',
                               'fp32_exact': 'fp32-input MFMA for every product'}[precision],
            'data': 'synthetic (Zipf two-domain sequences)',
            'config': {'workload': f'{name}: {cfg["label"]}', 'n_item_a': cfg['n_a'], 'n_item_b': cfg['n_b'],
                       'd': cfg['d'], 'seq_len': cfg['L'], 'batch_per_gpu': B_local, 'global_batch': B_global,
                       'train_sequences': int(n_rows), 'len_rec': 10, 'dropout': 0.2, 'parallelism': par},
            'loss': round(loss, 5) if math.isfinite(loss) else None, 'n_params': n_params,
            'host_prep': {'launch_counts_ms_per_step': round(host_counts_ms, 3),
                          'note': 'host data prep, outside the timed region (SURVEY §8(d)): the step\'s launch sizes '
                                  'counted from the batch\'s host copy by the data pipeline (Trainer.launch_counts); '
                                  'batches are staged in HBM before timing'},
            'roofline': roof, 'roofline_hbm': hb}


if __name__ == '__main__':
    main()
