"""Implied extents of every buffer a c2dsr_raw op WRITES (an undersized output tensor handed
to a raw op must raise, not be written past its end).  tools/gen_torch_ops.py turns each entry into a check before
the launch: the bytes from the tensor's data pointer to the end of its storage must cover the extent.

EXTENTS[op][param] = a C++ expression over the op's scalar parameters (as passed: int64_t / double) giving the
extent in ELEMENTS of the pointee type (float, int, int64_t, double, short), or in BYTES for a ``void*`` buffer.
Helpers: ``HAS(p)`` — pointer argument p is given; ``SPAN(rows, ld, cols)`` — a row-major [rows][cols] block with
row stride ld; the library's own size queries (c2dsr_*_workspace, c2dsr_attn_psave_floats, …).

UNCHECKED[op][param] = why no extent follows from the scalars: the rows written are named by device-side data
(a graph plan, compact row offsets, a row map) — those buffers are sized by the stage operators of c2dsr::, which
derive and check every extent from their tensors (csrc_torch/stage_ops.cpp, encoder_ops.cpp, losshead_ops.cpp).
"""

ROWS = 'rows * d'

EXTENTS = {
    'embed_fwd': {'X': 'n_rows * d', 'err': '1'},
    'embed_fwd_rows': {'X': '(nq + nk) * d', 'err': '1'},
    'index_check': {'err': '1'},
    'index_plan': {'plan': 'plan_bytes', 'err': '1'},
    'index_plans': {'err': '1'},
    'embed_bwd_planned': {'G': 'n_items * d', 'gP': 'n_pos * d', 'gXin': 'n_rows * d', 'workspace': 'ws_bytes'},
    'embed_fwd_b16': {'X': 'n_rows * d', 'err': '1'},
    'embed_bwd_planned_b16': {'G': 'n_items * d * 2', 'gP': 'n_pos * d', 'workspace': 'ws_bytes'},
    'embed_bwd_planned_rows': {'G': 'n_items * d', 'gP': 'n_pos * d', 'workspace': 'ws_bytes'},
    'embed_bwd': {'G': 'n_items * d', 'gP': 'n_pos * d', 'gXin': 'n_rows * d', 'workspace': 'ws_bytes'},
    'gemm': {'C': 'SPAN(M, ldc, N)'},
    'colsum': {'out': 'N', 'workspace': 'c2dsr_colsum_workspace((int)M, (int)N)'},
    'wcolsum': {'out': 'N', 'workspace': 'c2dsr_colsum_workspace((int)M, (int)N)'},
    'attn_fwd': {'out': 'B * L * d', 'Psave': 'c2dsr_attn_psave_floats((int)B, (int)L, (int)d, (int)H)'},
    'attn_bwd': {'dqkv': 'B * L * 3 * d'},
    'attn_bwd_b16': {'dqkv': 'B * L * 3 * d * 2'},
    'attn_fwd_rows': {'Psave': 'B * H * 4096'},
    'add_ln_fwd': {'xsave': ROWS, 'y': ROWS, 'mean': 'rows', 'rstd': 'rows'},
    'ln_bwd': {'dx': ROWS, 'db_out': ROWS, 'dgw': 'd', 'dgb': 'd', 'workspace': 'c2dsr_ln_bwd_workspace((int)d)'},
    'add_dropout': {'y': 'n'},
    'add_ln2_fwd': {'xsave': ROWS, 'y': ROWS, 'st': '4 * rows'},
    'ln2_bwd': {'dx': ROWS, 'db_out': ROWS, 'dgw2': 'd', 'dgb2': 'd', 'dgwF': 'd', 'dgbF': 'd',
                'workspace': 'c2dsr_ln2_bwd_workspace((int)d)'},
    'ln_reduce2': {'dgw2': 'HAS(dgw2) ? d : 0', 'dgb2': 'HAS(dgb2) ? d : 0', 'dgwF': 'HAS(dgwF) ? d : 0',
                   'dgbF': 'HAS(dgbF) ? d : 0', 'dgw1': 'HAS(dgw1) ? d : 0', 'dgb1': 'HAS(dgb1) ? d : 0'},
    'relu_drop_bwd': {'dx': 'n'},
    'pool_weights': {'w': 'B * L'},
    'pool_fwd': {'out': 'B * d'},
    'pool_bwd': {'dh': 'B * L * d'},
    'pool2_fwd': {'out1': 'B * d', 'out2': 'B * d'},
    'pool2_bwd': {'dh': '(HAS(idx) ? n_rows : B * L) * d'},
    'compact_valid': {'idx': 'M', 'inv': 'M', 'tc': 'M', 'counts': '2',
                      'ws': '(int64_t)c2dsr_compact_workspace((int)M, 1) / 4', 'err': '1'},
    'need_rows': {'idx': 'n_sets * B * L', 'inv': 'n_sets * B * L', 'count': 'n_sets', 'off': 'n_sets * (B + 1)',
                  'ws': '(int64_t)c2dsr_compact_workspace((int)(B * L), (int)n_sets) / 4'},
    'pad_rows': {'idx': 'n_sets * B * L', 'inv': 'n_sets * B * L', 'count': 'n_sets', 'off': 'n_sets * (B + 1)',
                 'ws': '(int64_t)c2dsr_compact_workspace((int)(B * L), (int)n_sets) / 4'},
    'combine_rows': {'dst': 'M * d'},
    'gather_rows': {'dst': 'n * d'},
    'expand_rows': {'dst': 'M * d'},
    'rowdot': {'out': 'SPAN(M, ldo, 1)'},
    'mi_scores': {'S': '4 * B'},
    'mi_loss': {'loss_mi': '1', 'ds': '4 * B'},
    'rec_gather': {'Hcat': '2 * B * R * d', 'Hpad': '2 * B * R * d'},
    'rec_gather_compact': {'Hpad': '2 * B * R * d', 'Hc': 'Mv * d', 'img': 'M_pad * d * (split ? 2 : 1) * 2'},
    'rec_targets': {'tcat': '2 * B * R'},
    'rec_scatter': {'dhs': 'HAS(dhs_map) ? 0 : B * L * d', 'dhx': 'HAS(dhx_map) ? 0 : B * L * d'},
    'ce_fwd': {'lse': 'M', 'loss_row': 'M'},
    'ce_bwd': {'logits': 'SPAN(M, ld, ncol)'},
    'outer_add': {'out': 'SPAN(M, ldo, d)'},
    'loss_partials': {'vec': '8', 'workspace': '(int64_t)c2dsr_loss_partials_workspace((int)BR)'},
    'loss_finalize': {'out3': '3', 'coefA': '2', 'coefB': '2'},
    'loss_accumulate': {'acc3': '3'},
    'scale_ds': {'ds': 'n'},
    'rowscale': {'out': 'n'},
    'bilinear_ds': {'dx1a': 'B * d', 'dx1b': 'B * d', 'dUa': '2 * B * d', 'dUb': '2 * B * d'},
    'f32_to_bf16': {'y': 'n * 2'},
    'ce_bias2': {'bias2': 'n_pad'},
    'ce_fused_fwd': {'part_m': 'n_split * M', 'part_s': 'n_split * M', 'lse': 'M', 'lse2': 'M', 'loss_row': 'M'},
    'ce_fused_fwd_u': {'part_m': 'n_split * M', 'part_s': 'n_split * M', 'Up': 'n_split * M * D', 'lse': 'M',
                       'lse2': 'M', 'loss_row': 'M'},
    'ce_dh_from_u': {'dH': 'M * D'},
    'ce_row_weights': {'rw': 'M_pad', 't32': 'M_pad', 'crow': 'M_pad', 'dpad': 'M'},
    'ce_fused_dh': {'dHp': 'n_split * M * D'},
    'ce_dh_combine': {'dH': 'M * D'},
    'ce_fused_dw': {'dWp': 'n_rsplit * n * D', 'dbp': 'n_rsplit * n'},
    'ce_onehot_dw_planned': {'gW': 'n * D', 'gb': 'n', 'workspace': 'ws_bytes'},
    'ce_onehot_dw': {'gW': 'n * D', 'gb': 'n', 'workspace': 'ws_bytes'},
    'ce_rows': {'lse': 'M', 'lse2': 'M', 'loss_row': 'M'},
    'f32_split_bf16': {'out': 'rows_out * 2 * D * 2'},
    'ce3_fused_fwd_u': {'part_m': 'n_split * M', 'part_s': 'n_split * M', 'Up': 'n_split * M * D', 'lse': 'M',
                        'lse2': 'M', 'loss_row': 'M'},
    'ce3_fused_dw': {'dWp': '(n_rsplit > 0 ? n_rsplit : 1) * n * D', 'dbp': '(n_rsplit > 0 ? n_rsplit : 1) * n'},
    'ce3b_fused_fwd_u': {'part_m': 'n_split * M', 'part_s': 'n_split * M', 'Up': 'n_split * M * D', 'lse': 'M',
                         'lse2': 'M', 'loss_row': 'M'},
    'ce3b_fused_dw': {'dWp': '(n_rsplit > 0 ? n_rsplit : 1) * n * D', 'dbp': '(n_rsplit > 0 ? n_rsplit : 1) * n'},
    'ce3_fused_dw_sk': {'gW': 'n * D', 'gb': 'n', 'ws': 'ws_bytes'},
    'ce3b_fused_dw_sk': {'gW': 'n * D', 'gb': 'n', 'ws': 'ws_bytes'},
    'sum_parts': {'out': 'n'},
    'selftest_tr': {'out': '64 * 16'},
    'adamw': {'p': 'n', 'fresh': 'n', 'accum': 'n', 'm': 'n', 'v': 'n', 'vmax': 'n'},
    'rgemm': {'C': 'SPAN(M, ldc, N)'},
    'rgemm_aux': {'C': 'SPAN(M, ldc, N)'},
    'rgemm_aux_b16a': {'C': 'SPAN(M, ldc, N)'},
    'rgemm_x3': {'C': 'SPAN(M, ldc, N)'},
    'rgemm_x3f': {'C': 'SPAN(M, ldc, N)'},
    'rgemm_x3_relu_guard': {'C': 'SPAN(M, ldc, N)', 'workspace': 'ws_bytes'},
    'wgemm_x3': {'dW': 'N * D', 'db': 'N', 'part': '(int64_t)c2dsr_wgemm_workspace((int)N)'},
    'wgemm_x3_multi': {'dW': 'N * D', 'db': 'N', 'part': '(int64_t)c2dsr_wgemm_workspace((int)N)'},
    'wgemm': {'dW': 'N * D', 'db': 'N', 'part': '(int64_t)c2dsr_wgemm_workspace((int)N)'},
    'wgemm_b16y': {'dW': 'N * D', 'db': 'N', 'part': '(int64_t)c2dsr_wgemm_workspace((int)N)'},
    'wgemm_multi': {'dW': 'N * D', 'db': 'N', 'part': '(int64_t)c2dsr_wgemm_workspace((int)N)'},
    'to_bf16': {'y': 'R * Cc * 2'},
    'eval_rank': {'rank': 'B'},
    'rank_metrics': {'sums': '8'},
}

_PLAN = 'the output rows are named by the device-side SpMM work plan (row count not an argument; ' \
        'c2dsr::gcn_* check the graph against the table)'
_ROWS = 'rows from the device-side compact offsets (q_off / k_off); c2dsr::encoder_pass sizes them'
UNCHECKED = {
    'gcn_spmm': {'part': _PLAN, 'Y': _PLAN, 'Y2': _PLAN},
    'gcn_spmm_b16': {'part': _PLAN, 'Y': _PLAN, 'Y2': _PLAN},
    'attn_fwd_rows': {'out': _ROWS},
    'attn_bwd_rows': {'dq': _ROWS, 'dkv': _ROWS},
}
