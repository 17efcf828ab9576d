"""torch.autograd bindings of the HIP kernels (every op here launches our own
gfx950 kernels through the C ABI; torch only allocates memory and orders streams).

Gradients of the model's own (flattened) parameters are written straight into
their ``.grad`` buffers by the kernels (accumulating, like AccumulateGrad would),
so autograd never materialises a second copy of a table-sized gradient.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.autograd import Function

from ._lib import HipLibError, error_word, lib, stream, require_device, stage_ops
from .dp import notify_lookup, notify_rows, notify_table, row_cuts

# precision modes: FP32 = the reference's precision (fp32 results; products on split-bf16 MFMAs where a kernel
# exists — ce3.hip —, exact fp32-input MFMA elsewhere), BF16 = bf16 operands with fp32 accumulation,
# FP32_EXACT = exact fp32-input MFMA for every product (materialised logits; the A/B check of FP32)
FP32, BF16, FP32_EXACT = 0, 1, 2


def flat_keys(keys):
    """[(k0, k1), …] → [k0, k1, …] (the stage operators' int[] keys)"""
    return [int(v) for k in keys for v in k]


def _grad_target(param):
    """The buffer a kernel may accumulate a parameter's gradient into, or None."""
    if param is None or not param.requires_grad:
        return None
    g = param.grad
    if g is None:
        param.grad = torch.zeros_like(param)
        g = param.grad
    return g


# ----------------------------------------------------------------------------- GEMM helpers
def gemm(A, B, C, *, M, N, K, transA=0, transB=0, lda=None, ldb=None, ldc=None, alpha=1.0, beta=0.0, bias=None,
         relu_drop=None, precision=FP32, split_k=0, rowmap=None):
    """C = alpha·op(A)·op(B) + beta·C + bias (see include/c2dsr.h:c2dsr_gemm)."""
    if lda is None:
        lda = M if transA else K
    if ldb is None:
        ldb = K if transB else N
    if ldc is None:
        ldc = N
    k0 = k1 = 0
    p = 0.0
    row_base = 0
    epi = 0
    if relu_drop is not None:
        epi = 1
        (k0, k1), p, row_base = relu_drop[:3]
        if len(relu_drop) > 3:
            rowmap = relu_drop[3]
    lib('c2dsr_gemm', transA, transB, M, N, K, A, lda, B, ldb, C, ldc, float(alpha), float(beta), bias, epi, k0, k1,
        float(p), int(row_base), rowmap, precision, split_k, stream())
    return C


def colsum(X, M, N, ldx, out, alpha=1.0, beta=1.0):
    """out[n] = beta·out[n] + alpha·Σ_m X[m·ldx + n]"""
    ws = torch.empty(lib.raw('c2dsr_colsum_workspace')(M, N), dtype=torch.uint8, device=out.device)
    lib('c2dsr_colsum', X, M, N, ldx, float(alpha), float(beta), out, ws, stream())


def rgemm_ok(M, N, K):
    return bool(lib.raw('c2dsr_rgemm_supported')(M, N, K))


def rg_kind(precision, M, N, K):
    """The row-streaming projection kernel (csrc/rgemm.hip) for this precision and shape: 'b16' (bf16
    operands), 'x3' (split-bf16 operands: the fp32 mode) or None (the tiled GEMM, exact fp32 MFMA)."""
    if precision == BF16 and rgemm_ok(M, N, K):
        return 'b16'
    if precision == FP32 and bool(lib.raw('c2dsr_rgemm_x3_supported')(M, N, K)):
        return 'x3'
    return None


def wg_kind(precision, T, N, D):
    """The weight-gradient kernel (c2dsr_wgemm / _x3) for this precision and shape, like rg_kind."""
    if precision in (BF16, FP32) and wgemm_ok(T, N, D):
        return 'b16' if precision == BF16 else 'x3'
    return None


def to_bf16(X, trans=False):
    """bf16 copy of a 2-D fp32 matrix (transposed if asked)."""
    R, Cc = X.shape
    y = torch.empty((Cc, R) if trans else (R, Cc), device=X.device, dtype=torch.bfloat16)
    lib('c2dsr_to_bf16', X, R, Cc, X.stride(0), int(trans), y, stream())
    return y


# bf16 images of the projection weights, made once per weight update: the three sequence-encoder
# passes through one SelfAttention share weights, and every forward / backward product re-used to
# convert them.  Valid while neither the fused optimizer (WEIGHTS.epoch, bumped per step) nor a torch
# in-place op (W._version) has written the weight since.
# After a bump, the first request converts every image used in the previous epoch in ONE launch
# (c2dsr_to_bf16_multi, rewriting the previous images in place) instead of one small launch per image.
class _WeightImages:
    def __init__(self):
        self.epoch = 0
        self.cache = {}  # key -> (tag, image)
        self.known = {}  # key -> (W, image) of the previous epoch: refreshed together on the next request

    def bump(self):
        """After an optimizer step: re-convert every image used this epoch now, behind the update on the stream
        (the host does it while the GPU runs the optimizer, not at the first projection of the next forward)."""
        self.epoch += 1
        self.known = {k: (v[2], v[1]) for k, v in self.cache.items()}  # the images used this epoch
        self.cache.clear()
        if self.known:
            self._refresh_known()

    LAYOUT = {None: 0, 'split': 1, 'frag': 2, 'b16frag': 3, 'norm2': 4}  # c2dsr::weight_images' layout codes

    def _refresh_known(self):
        done = [(key, W, y) for key, (W, y) in self.known.items() if key[3] in self.LAYOUT]
        if done:  # one stage operator: a multi-matrix launch per layout
            stage_ops().weight_images([W for _, W, _ in done], [y for _, _, y in done], [int(k[2]) for k, _, _ in done],
                                      [self.LAYOUT[k[3]] for k, _, _ in done])
        for key, W, y in done:
            self.cache[key] = ((self.epoch, W._version), y, W)
        self.known = {}

    def get(self, W, trans, layout=None):
        """layout None: bf16 image; 'b16frag': the bf16 image in rg_kernel's fragment order; 'split': split image
        hi ‖ lo; 'frag': the split image in rg3's fragment order; 'norm2': the squared row norms ‖W[r]‖² (the guarded
        linear1's threshold)."""
        key = (W.data_ptr(), tuple(W.shape), bool(trans), layout)
        tag = (self.epoch, W._version)
        if key not in self.cache and key in self.known:
            self._refresh_known()
        hit = self.cache.get(key)
        if hit is not None and hit[0] == tag:
            return hit[1]
        if layout == 'norm2':  # ‖W[r]‖² [R] (c2dsr_row_sqnorm_multi: one wave per row, fixed order)
            y = torch.empty(W.shape[0], device=W.device, dtype=torch.float32)
            stage_ops().weight_images([W], [y], [0], [4])
        elif layout == 'b16frag':
            R, Cc = W.shape
            rows, cols = (Cc, R) if trans else (R, Cc)
            y = torch.zeros(-(-rows // 32) * 32, cols, device=W.device, dtype=torch.bfloat16)
            desc = np.asarray([W.data_ptr(), y.data_ptr(), R, Cc, W.stride(0), int(trans)], dtype=np.int64)
            lib('c2dsr_to_bf16_frag_multi', desc, 1, stream())
        else:
            y = to_bf16(W, trans) if layout is None else to_split_bf16(W, trans, frag=layout == 'frag')
        self.cache[key] = (tag, y, W)
        return y


WEIGHTS = _WeightImages()


def weight_bf16(W, trans=False):
    return WEIGHTS.get(W.detach(), trans)


def weight_img(W, kind, trans=False):
    """The operand image of a projection weight for a rg_kind kernel, in the row-streaming kernels' fragment order
    (rgemm(..., frag=True)): bf16 ('b16') or split hi ‖ lo ('x3'); or the split image as rows [R][2C] ('x3row');
    transposed ([C][…]) if asked."""
    layout = {'b16': 'b16frag', 'x3': 'frag', 'x3row': 'split'}[kind]
    return WEIGHTS.get(W.detach(), trans, layout=layout)


def to_split_bf16(X, trans=False, frag=False):
    """Split-bf16 image of a 2-D fp32 matrix: [R][2C] with row = hi ‖ lo ([C][2R] if transposed); frag: the same
    values in c2dsr_rgemm_x3f's fragment order, rows padded to a multiple of 16 (zero)."""
    R, Cc = X.shape
    rows, cols = (Cc, R) if trans else (R, Cc)
    if frag:
        y = torch.zeros(-(-rows // 16) * 16, 2 * cols, device=X.device, dtype=torch.bfloat16)
    else:
        y = torch.empty(rows, 2 * cols, device=X.device, dtype=torch.bfloat16)
    desc = np.asarray([X.data_ptr(), y.data_ptr(), R, Cc, X.stride(0), int(trans)], dtype=np.int64)
    lib('c2dsr_to_split_bf16_frag_multi' if frag else 'c2dsr_to_split_bf16_multi', desc, 1, stream())
    return y


AUX_ACC, AUX_MASK, AUX_ACC_MAP = 1, 2, 3


def rgemm(A, Bb, C, *, M, N, K, alpha=1.0, beta=0.0, bias=None, relu_drop=None, aux_mode=0, aux=None, aux_scale=0.0,
          rowmap=None, auxmap=None, x3=False, frag=False):
    """C = alpha·A·Bbᵀ + beta·C + bias with A fp32 [M, K], Bb bf16 [N, K] (c2dsr_rgemm); aux_mode
    AUX_ACC: C += aux (aux may be C itself), AUX_MASK: C = aux > 0 ? C·aux_scale : 0 (c2dsr_rgemm_aux).
    x3: Bb is the split image [N, 2K] and the products run on split-bf16 operands (c2dsr_rgemm_x3); frag: Bb is
    the (bf16 or split) image in the kernel's fragment order (weight_img; c2dsr_rgemm_x3f, or ldb = 0)."""
    k0 = k1 = 0
    p = 0.0
    row_base = 0
    epi = 0
    if relu_drop is not None:
        epi = 1
        (k0, k1), p, row_base = relu_drop[:3]
        if len(relu_drop) > 3:
            rowmap = relu_drop[3]
    if x3:
        if A.dtype != torch.float32 or Bb.dtype != torch.bfloat16 or Bb.shape[-1] != 2 * K:
            raise TypeError(f'rgemm x3: A must be fp32 and Bb a split image [N, 2K] (got A {A.dtype}, Bb {Bb.dtype} '
                            f'{tuple(Bb.shape)})')
        if frag:
            lib('c2dsr_rgemm_x3f', M, N, K, A, K, Bb, C, N, float(alpha), float(beta), bias, epi, k0, k1, float(p),
                int(row_base), rowmap, int(aux_mode), aux, auxmap, float(aux_scale), stream())
        else:
            lib('c2dsr_rgemm_x3', M, N, K, A, K, Bb, 2 * K, C, N, float(alpha), float(beta), bias, epi, k0, k1,
                float(p), int(row_base), rowmap, int(aux_mode), aux, auxmap, float(aux_scale), stream())
    elif A.dtype == torch.bfloat16:  # the attention backward's bf16 dqkv (in_proj dX; c2dsr_rgemm_aux_b16a)
        if epi or aux_mode == AUX_MASK:
            raise HipLibError('rgemm: bf16 A supports no epilogue / mask mode')
        lib('c2dsr_rgemm_aux_b16a', M, N, K, A, K, Bb, 0 if frag else K, C, N, float(alpha), float(beta), bias,
            int(aux_mode), aux, auxmap, stream())
    elif aux_mode:
        lib('c2dsr_rgemm_aux', M, N, K, A, K, Bb, 0 if frag else K, C, N, float(alpha), float(beta), bias, epi, k0, k1,
            float(p), int(row_base), rowmap, int(aux_mode), aux, auxmap, float(aux_scale), stream())
    else:
        lib('c2dsr_rgemm', M, N, K, A, K, Bb, 0 if frag else K, C, N, float(alpha), float(beta), bias, epi, k0, k1,
            float(p), int(row_base), rowmap, stream())
    return C


_GUARD_WS = {}  # device -> the guarded producer's workspace (c2dsr_rgemm_guard_workspace)


def rgemm_relu_guard(A, Wimg, W, C, *, M, N, K, bias, relu_drop, frag=False, wn2=None):
    """C = drop(relu(A·Wᵀ + bias)) in the fp32 mode (c2dsr_rgemm_x3_relu_guard): split-bf16 products with every
    pre-activation within the split error bound of zero recomputed exactly from the fp32 A and W (linear1: its
    ReLU's sign decisions select the dy·x terms of the weight gradient).  frag: Wimg is the fragment-ordered image;
    wn2: ‖W[c]‖² [N] kept per weight update (weight_norm2), else computed in the call."""
    (k0, k1), p, row_base = relu_drop[:3]
    rowmap = relu_drop[3] if len(relu_drop) > 3 else None
    if A.dtype != torch.float32 or W.dtype != torch.float32 or Wimg.shape[-1] != 2 * K:
        raise TypeError('rgemm_relu_guard: fp32 A and W, split image [N, 2K]')
    wsb = int(lib.raw('c2dsr_rgemm_guard_workspace')(M, N))
    ws = _GUARD_WS.get(A.device)
    if ws is None or ws.numel() < wsb:  # zeroed once: every call leaves its block flags cleared
        ws = _GUARD_WS[A.device] = torch.zeros(max(wsb, 1 << 20), device=A.device, dtype=torch.uint8)
    lib('c2dsr_rgemm_x3_relu_guard', M, N, K, A, K, Wimg, 0 if frag else 2 * K, W, wn2, C, N, bias, k0, k1, float(p),
        int(row_base), rowmap, ws, ws.numel(), stream())
    return C


RELU_GUARD = True  # linear1 of the fp32 mode on the guarded split kernel (see LinearFn.forward)


def relu_guard_ok(M, N, K):
    return K == 256 and N % 4 == 0 and bool(lib.raw('c2dsr_rgemm_x3_supported')(M, N, K))


def wgemm_ok(T, N, D):
    return bool(lib.raw('c2dsr_wgemm_supported')(T, N, D))


class WGradBatch:
    """The projection weight-gradient products of one training backward, deferred and grouped per weight: a
    SelfAttention module that several encoder passes used (attn_share: the share pass and both negative
    passes) gets ONE c2dsr_wgemm_multi product over all its passes' rows instead of one per pass (one set of
    split partials and one fixed-order sum instead of three).  Flushed when the last embedding backward
    (``lookups`` of them) finishes — before the data-parallel hook issues the dense range — or by the
    trainer after the backward."""

    def __init__(self, lookups):
        self.groups = {}
        self.lookups_left = lookups

    def add(self, dY, X, dW, db, T, N, D, x3=False):
        key = (dW.data_ptr(), N, D, dY.dtype, None if db is None else db.data_ptr(), x3)
        g = self.groups.setdefault(key, [dW, db, []])
        g[2].append((dY, X, T))

    def lookup_done(self):
        self.lookups_left -= 1
        if self.lookups_left == 0:
            self.flush()

    def flush(self):
        """All groups' products in one stage operator (c2dsr::wgrad_groups: per group, four segments per product)."""
        if not self.groups:
            return
        dYs, Xs, gid, dWs, dbs, x3s = [], [], [], [], [], []
        for g, ((_, N, D, dt, _, x3), (dW, db, segs)) in enumerate(self.groups.items()):
            for dY, X, T in segs:
                dYs.append(dY.reshape(-1, N)[:T])
                Xs.append(X.reshape(-1, D)[:T])
                gid.append(g)
            dWs.append(dW.view(N, D))
            dbs.append(db)
            x3s.append(int(x3))
        stage_ops().wgrad_groups(dYs, Xs, gid, dWs, dbs, x3s)
        self.groups = {}


WBATCH = None  # the active WGradBatch (Trainer.train_batch, bf16 / fp32 mode), else None


def wgemm(dY, X, dW, *, T, N, D, beta=1.0, db=None, defer=True, x3=False):
    """dW[N, D] = beta·dW + dYᵀ·X over T rows and (db given) db[N] = beta·db + Σ_t dY[t]
    (c2dsr_wgemm, deterministic split-t partials; x3: split-bf16 products, c2dsr_wgemm_x3).  With a
    WGradBatch active (and beta = 1) the product is deferred into it."""
    if x3 and (dY.dtype != torch.float32 or X.dtype != torch.float32):
        raise TypeError(f'wgemm x3: fp32 operands only (got dY {dY.dtype}, X {X.dtype})')
    if defer and WBATCH is not None and beta == 1.0 and dY.is_contiguous() and X.is_contiguous():
        WBATCH.add(dY, X, dW, db, T, N, D, x3)
        return
    ws = torch.empty(lib.raw('c2dsr_wgemm_workspace')(N), dtype=torch.uint8, device=dW.device)
    if x3:
        name = 'c2dsr_wgemm_x3'
    else:
        name = 'c2dsr_wgemm_b16y' if dY.dtype == torch.bfloat16 else 'c2dsr_wgemm'
    lib(name, T, N, D, dY, N, X, D, float(beta), dW, db, ws, stream())


class ResidualLink:
    """Joins the two consumers of a post-norm encoder layer's input x — the layer's first projection and
    the residual branch of its LayerNorm (models/encoders.py:23-27 → transformer.py: x = norm(x + block(x))).
    The LayerNorm backward parks its gradient w.r.t. x here instead of returning it; the projection's dX
    product then accumulates onto it in its epilogue, so autograd never adds the two in a separate pass."""

    def __init__(self, inv=None):
        self.grad = None
        self.inv = inv  # the LN ran on a row subset: its parked gradient is compact, expanded here (RowSet.inv)


class FFLink:
    """Joins linear1 (drop(relu(.)) epilogue) and linear2 of a feed-forward block: when linear2's dX
    product applied the drop(relu) backward in its epilogue (mask = linear2's input > 0), linear1
    receives an already-masked gradient."""

    def __init__(self, p):
        self.p = p
        self.premasked = False


class LinearFn(Function):
    """y = x·Wᵀ + b  [optionally drop(relu(.))]  — nn.Linear / TransformerEncoderLayer linear1, linear2,
    in_proj, out_proj (models/encoders.py:23-27 → torch transformer.py).  bf16 mode at d = 256-multiples:
    the row-streaming MFMA kernels (csrc/rgemm.hip); otherwise the tiled GEMM (csrc/gemm.hip).
    res: ResidualLink (this projection reads the layer input; its dX accumulates onto the parked LN
    gradient).  ff: FFLink — role 'in' for linear1 (the relu-drop producer), 'out' for linear2."""

    @staticmethod
    def forward(ctx, x, W, b, precision, relu_drop, res=None, ff=None, ff_role=None):
        require_device(x)
        N, K = W.shape
        M = x.numel() // K
        y = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
        kind = rg_kind(precision, M, N, K)
        if kind == 'x3' and relu_drop is not None:
            # the ReLU producer (linear1): its sign decisions select which gradient terms exist, so a
            # pre-activation within the split product's rounding (~1e-5 relative) of zero would flip a whole
            # dy·x term of the weight gradient (tools/fp32_diag.py: 2e-3 vs 1.6e-5 with this product exact).
            # RELU_GUARD (default): split products, every pre-activation inside the split error bound recomputed as
            # a k-ordered fp32 FMA chain (c2dsr_rgemm_x3_relu_guard; the order decides the reference C2 step's
            # ties: a float64-exact product misses it by 1.2e-4, tools/linear1_emu.py) — 105 → 60 µs at 57k rows;
            # otherwise the exact fp32-input MFMA GEMM
            kind = None
            if RELU_GUARD and relu_guard_ok(M, N, K):
                rgemm_relu_guard(x, weight_img(W, 'x3'), W, y, M=M, N=N, K=K, bias=b, relu_drop=relu_drop,
                                 frag=True, wn2=WEIGHTS.get(W.detach(), False, layout='norm2'))
                kind = 'guard'
        if kind == 'guard':
            pass
        elif kind:
            rgemm(x, weight_img(W, kind), y, M=M, N=N, K=K, bias=b, relu_drop=relu_drop, x3=kind == 'x3',
                  frag=True)
        else:
            gemm(x, W, y, M=M, N=N, K=K, transB=1, bias=b, relu_drop=relu_drop, precision=precision)
        ctx.save_for_backward(x, W, y if relu_drop is not None else None)
        ctx.b = b
        ctx.precision = precision
        ctx.relu_p = relu_drop[1] if relu_drop is not None else None
        ctx.res, ctx.ff, ctx.ff_role = res, ff, ff_role
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, y = ctx.saved_tensors
        dx = linear_backward(ctx, x, W, y, dy, ctx.needs_input_grad[0])
        return dx, None, None, None, None, None, None, None


def linear_backward(ctx, x, W, y, dy, need_dx):
    """The backward of y = x·Wᵀ + b [drop(relu)] (LinearFn.backward; QKVAttnFn's in_proj part).  ctx carries
    b, precision, relu_p, res, ff, ff_role.  dy may be bf16 (the attention's dqkv): then the fused bf16-mode
    kernels are taken, which read it without conversion."""
    N, K = W.shape
    M = x.numel() // K
    dy = dy.contiguous()
    if ctx.relu_p is not None and not (ctx.ff is not None and ctx.ff.premasked):
        d2 = torch.empty_like(dy)
        lib('c2dsr_relu_drop_bwd', dy, y, dy.numel(), float(ctx.relu_p), d2, stream())
        dy = d2
    dx = None
    if need_dx:
        kind = rg_kind(ctx.precision, M, K, N)
        fused = kind is not None
        x3 = kind == 'x3'
        Wt = weight_img(W, kind, trans=True) if fused else None
        park = ctx.res.grad if ctx.res is not None else None
        if ctx.res is not None:
            ctx.res.grad = None
        sub = park is not None and ctx.res.inv is not None  # parked gradient of a row subset
        if sub and not fused:  # compact rows → full, zeros elsewhere
            full = torch.empty_like(x)
            lib('c2dsr_expand_rows', park, ctx.res.inv, M, K, full, stream())
            park, sub = full, False
        if sub:  # dx = dy·W + the parked rows, read through the row map
            dx = torch.empty_like(x)
            rgemm(dy, Wt, dx, M=M, N=K, K=N, aux_mode=AUX_ACC_MAP, aux=park, auxmap=ctx.res.inv, x3=x3, frag=True)
        elif fused and park is not None:  # dx = parked LN gradient + dy·W, in place
            dx = park
            rgemm(dy, Wt, dx, M=M, N=K, K=N, aux_mode=AUX_ACC, aux=dx, x3=x3, frag=True)
        elif fused and ctx.ff is not None and ctx.ff_role == 'out':  # linear1's drop(relu) backward here
            dx = torch.empty_like(x)
            rgemm(dy, Wt, dx, M=M, N=K, K=N, aux_mode=AUX_MASK, aux=x, aux_scale=1.0 / (1.0 - ctx.ff.p), x3=x3,
                  frag=True)
            ctx.ff.premasked = True
        elif fused:
            dx = torch.empty_like(x)
            rgemm(dy, Wt, dx, M=M, N=K, K=N, x3=x3, frag=True)
        elif park is not None:
            dx = park
            gemm(dy, W, dx, M=M, N=K, K=N, beta=1.0, precision=ctx.precision)
        else:
            dx = torch.empty_like(x)
            gemm(dy, W, dx, M=M, N=K, K=N, precision=ctx.precision)
    gW = _grad_target(W)
    gb = _grad_target(ctx.b)
    wk = wg_kind(ctx.precision, M, N, K) if dy.dtype == torch.float32 or ctx.precision == BF16 else None
    if gW is not None and wk:
        wgemm(dy, x, gW, T=M, N=N, D=K, db=gb, x3=wk == 'x3')  # bias gradient from the same dY chunks
        gb = None
    elif gW is not None:
        gemm(dy, x, gW, M=N, N=K, K=M, transA=1, lda=N, ldb=K, beta=1.0, precision=ctx.precision)
    if gb is not None:
        colsum(dy, M, N, N, gb)
    return dx




def linear(x, W, b, precision=FP32, relu_drop=None, res=None, ff=None, ff_role=None):
    return LinearFn.apply(x.contiguous(), W, b, precision, relu_drop, res, ff, ff_role)


# ----------------------------------------------------------------------------- row subsets
# the bits of the device index error word (include/c2dsr.h C2DSR_IDX_ERR_*)
IDX_ERR_ITEM, IDX_ERR_POS, IDX_ERR_PLAN, IDX_ERR_TARGET = 1, 2, 4, 8


def index_error_message(bits):
    """The IndexError text for an error word: torch's own F.embedding message plus which lookup failed."""
    what = [n for b, n in ((IDX_ERR_ITEM, 'item index outside [0, n_item)'), (IDX_ERR_POS, 'position outside [0, len_max)'),
                           (IDX_ERR_PLAN, 'lookup index outside its table'),
                           (IDX_ERR_TARGET, 'target outside [0, n_item_x]')) if bits & b]
    return 'index out of range in self (' + '; '.join(what or [f'error word {bits:#x}']) + ')'


class HostCounts:
    """Small device int32 counts copied to pinned host memory behind the work that produces them, read
    on first use: the host blocks only if the device has not got that far yet, so the stream never
    drains the way an immediate ``.tolist()`` would make it."""

    def __init__(self, dev_counts, known=None, check=False, err_slot=None):
        """known: the same counts computed on the host from the batch's host copy (Trainer.host_counts) — then
        nothing is copied and nothing ever waits on the device; check: also copy the device counts and compare
        them with ``known`` at the first read (C2DSR_CHECK_COUNTS=1; raises on a mismatch).  err_slot: the slot
        holding the device's index error word after the batch's range checks (c2dsr::index_check, a batch without
        a host copy): nonzero raises IndexError at the first read, before any backward or optimizer launch."""
        self.err_slot = err_slot
        self.known = None if known is None else [int(v) for v in known]
        if self.known is not None and len(self.known) != dev_counts.numel():
            # counts prepared under other count_flags (model mode, seqs=None, …) would be read from wrong slots
            raise ValueError(f'{len(self.known)} host-prepared counts for {dev_counts.numel()} device count slots')
        self.vals = self.known if not check else None
        if self.vals is None:
            self.host = torch.empty(dev_counts.numel(), dtype=torch.int32, pin_memory=True)
            self.host.copy_(dev_counts, non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record()

    def __getitem__(self, i):
        if self.vals is None:
            self.ev.synchronize()
            self.vals = self.host.tolist()
            if self.err_slot is not None and self.vals[self.err_slot]:
                bits, self.vals = self.vals[self.err_slot], None
                error_word().zero_()
                raise IndexError(index_error_message(bits))
            if self.known is not None and self.known != self.vals:
                raise RuntimeError(f'host-computed counts {self.known} != device counts {self.vals}')
        return self.vals[i]


class RowSet:
    """The rows of one encoder pass the loss reads (c2dsr_need_rows) — or its padding rows, the attention's
    keys (c2dsr_pad_rows): idx [n] (ascending), inv [M] (compact index or -1).  The last encoder layer runs
    its row-wise part on these rows only.  ``n`` may be given as (HostCounts, slot), read when first needed."""

    def __init__(self, idx, inv, n, M, off=None):
        self.idx, self.inv, self.M = idx, inv, int(M)
        self.off = off  # [B + 1] compact index of each sequence's first row (c2dsr_need_rows / c2dsr_pad_rows)
        self._n = n

    @property
    def n(self):
        if isinstance(self._n, tuple):
            hc, q = self._n
            self._n = int(hc[q])
        return int(self._n)


class GatherRowsFn(Function):
    """[M, d] → [n, d] rows of a RowSet; backward scatters into zeros."""

    @staticmethod
    def forward(ctx, x, rs):
        d = x.shape[-1]
        out = torch.empty(rs.n, d, device=x.device, dtype=x.dtype)
        lib('c2dsr_gather_rows', x, d, rs.idx, rs.n, d, out, stream())
        ctx.rs, ctx.shape = rs, x.shape
        return out

    @staticmethod
    def backward(ctx, g):
        rs = ctx.rs
        full = torch.empty(ctx.shape, device=g.device, dtype=g.dtype)
        lib('c2dsr_expand_rows', g.contiguous(), rs.inv, rs.M, g.shape[-1], full, stream())
        return full, None


class ExpandRowsFn(Function):
    """[n, d] rows of a RowSet → [*shape] with zeros elsewhere; backward gathers."""

    @staticmethod
    def forward(ctx, xc, rs, shape):
        d = xc.shape[-1]
        out = torch.empty(shape, device=xc.device, dtype=xc.dtype)
        lib('c2dsr_expand_rows', xc, rs.inv, rs.M, d, out, stream())
        ctx.rs = rs
        return out

    @staticmethod
    def backward(ctx, g):
        rs = ctx.rs
        d = g.shape[-1]
        out = torch.empty(rs.n, d, device=g.device, dtype=g.dtype)
        lib('c2dsr_gather_rows', g.contiguous(), d, rs.idx, rs.n, d, out, stream())
        return out, None, None


def gather_rows_nograd(x, rs):
    d = x.shape[-1]
    out = torch.empty(rs.n, d, device=x.device, dtype=x.dtype)
    lib('c2dsr_gather_rows', x.detach(), d, rs.idx, rs.n, d, out, stream())
    return out


# ----------------------------------------------------------------------------- GCN (K1)
EAGER_GCN = True  # a table's GCN backward runs as soon as its last lookup's backward has filled the sink


class GradSink:
    """Dense gradient w.r.t. one GCN output table H, filled by every embedding lookup of H
    (deterministic segment sums) and consumed once by the GCN backward.

    The GCN backward of a table needs nothing but this sink (the table's gradient E.grad is written by it alone), so
    it runs as soon as the LAST lookup of H has run its backward (``lookup_done``, counting the lookups recorded since
    the propagation, ``uses``) instead of where autograd would schedule GCNFn's node — after every other node, since
    it was created first.  With data parallelism that issues each item table's collectives right after its own
    pass (dp.py: table B's under the backward of passes A and share, table A's under the share pass), instead of all
    three tables' at the end of the backward.  Same kernels on the same inputs: bit-identical gradients."""

    def __init__(self, n, d, device, state=None):
        self.n, self.d, self.device = n, d, device
        self.G = None
        self.state = state  # StepState: carries the data-parallel bucket hook (c2dsr_amd/dp.py)
        self.uses = 0      # lookups of H recorded (with a backward to come) since the propagation
        self.gcn = None    # (graph, n_gnn, p, keys, pad_row, E) of the propagation whose backward is pending
        self.ran = False   # that backward already ran (eagerly): GCNFn.backward has nothing left to do

    def buf(self):
        if self.G is None:
            self.G = torch.zeros(self.n, self.d, device=self.device, dtype=torch.float32)
        return self.G

    def propagated(self, gcn):
        self.uses, self.gcn, self.ran = 0, gcn, False

    def lookup_recorded(self):
        self.uses += 1

    def lookup_done(self):
        """One lookup of H finished its backward; the last one runs the table's GCN backward now."""
        self.uses -= 1
        if self.uses == 0 and self.gcn is not None and EAGER_GCN and self.gcn[5].grad is not None:
            args, self.gcn = self.gcn, None
            gcn_backward(self, *args)
            self.ran = True


class RowShard:
    """Row-sharded GCN propagation over ``world`` data-parallel ranks: rank r owns rows
    [r·c, (r+1)·c) of every propagated table, c = ⌈N/world⌉; tables are allocated with world·c rows (the tail
    beyond N is never written or read) so the blocks all-gather in place."""

    def __init__(self, rank, world, gather=None):
        from .dp import all_gather
        self.rank, self.world = rank, world
        self._gather = gather or all_gather
        self.pending = []

    def block(self, n):
        return (n + self.world - 1) // self.world

    def rows(self, n):
        c = self.block(n)
        return min(n, self.rank * c), min(n, (self.rank + 1) * c)

    def buffer(self, like):
        n, d = like.shape
        return torch.empty(self.block(n) * self.world, d, device=like.device, dtype=like.dtype)

    def gather(self, full):
        c = full.shape[0] // self.world
        return self._gather(full, full[self.rank * c:(self.rank + 1) * c])

    def wait(self):
        for w in self.pending:
            w.wait()
        self.pending = []


SPMM_SLICE = {}  # work-list pointer of a row-slice SpMM launch -> (rows, edges) (roofline accounting)


def spmm(graph, transposed, X, keys, p, mask_on_output, alpha, Z, beta, delta, pad_row, gamma, Y, Y2=None,
         rows=None, part=None):
    """Y = alpha·P + (beta + [i != pad]·delta)·Z + gamma·Y with P = A·drop(X) (or drop(Aᵀ·X)); see c2dsr_gcn_spmm.
    ``rows`` = (r0, r1): only output rows r0..r1 (the work items / split combines of those rows: the plan
    is sorted by row and a split row's pieces share its row, so a row range is a contiguous slice of both)."""
    work, n_work, split, n_split, n_slots, col, val = graph.plan(transposed)
    d = X.shape[1]
    if part is None:
        part = torch.empty(max(n_slots, 1), d, device=X.device, dtype=torch.float32)
    if rows is not None:
        w0, w1, s0, s1 = graph.row_slice(transposed, *rows)
        work, n_work, split, n_split = work[w0:w1], w1 - w0, split[s0:s1], s1 - s0
        if w1 > w0:  # roofline accounting of a row-slice launch (bench.py HbmTimer): its rows and edges
            rp = graph.host_rowptr(transposed)
            SPMM_SLICE[work.data_ptr()] = (rows[1] - rows[0], int(rp[rows[1]]) - int(rp[rows[0]]))
    name = 'c2dsr_gcn_spmm_b16' if X.dtype == torch.bfloat16 else 'c2dsr_gcn_spmm'  # bf16 tables: the C5 run
    lib(name, work, n_work, split, n_split, part, col, val, d, X, keys[0], keys[1], float(p),
        int(mask_on_output), float(alpha), Z, float(beta), float(delta), int(pad_row), float(gamma), Y, Y2, stream())
    return part


class GCNFn(Function):
    """H = mean(E, A·drop(E), A·drop(A·drop(E)), ...)  (models/encoders.py:42-48).
    Outputs (H, token): H is non-differentiable; the scalar token carries the
    dependency of every lookup of H back to this node.

    ``shard`` = a RowShard (data parallel): this rank propagates only its block of rows of
    every round (the SpMM's row slice: the same work items, so the same bits) and the blocks are all-gathered —
    synchronously for an intermediate round (the next round reads every row), asynchronously for H, whose
    handle ``shard.pending`` is waited on before H is first read (C2DSR.forward).  The backward is unchanged:
    each rank runs Aᵀ over its own lookup gradient and the flat-gradient exchange sums the ranks (dp.py)."""

    @staticmethod
    def forward(ctx, E, graph, n_gnn, p, keys, pad_row, sink, shard=None):
        require_device(E)
        inv = 1.0 / (n_gnn + 1)
        rows = None
        if shard is None or n_gnn == 0:  # the whole table: one stage operator (all rounds)
            work, _, split, _, n_slots, col, val = graph.plan(False)
            out = stage_ops().gcn_propagate(E, work, split, col, val, graph.n, n_slots, n_gnn, float(p),
                                            flat_keys(keys))
            ctx.graph, ctx.n_gnn, ctx.p, ctx.keys, ctx.pad_row, ctx.sink = graph, n_gnn, p, keys, pad_row, sink
            ctx.E = E
            sink.propagated((graph, n_gnn, p, keys, pad_row, E))
            ctx.mark_non_differentiable(out)
            ctx.set_materialize_grads(False)
            return out, torch.empty((), device=E.device)
        out_full = shard.buffer(E)
        out = out_full[:E.shape[0]]
        rows = shard.rows(E.shape[0])
        if n_gnn == 0:  # H = E
            spmm(graph, False, E, (0, 0), 0.0, 0, 0.0, E, 1.0, 0.0, -1, 0.0, out)
        h_prev = E
        for k in range(n_gnn):
            last = k == n_gnn - 1
            h_full = None
            if not last:
                h_full = shard.buffer(E) if rows is not None else torch.empty_like(E)
            h_k = None if last else h_full[:E.shape[0]]
            spmm(graph, False, h_prev, keys[k], p, 0, inv, E if k == 0 else None, inv, 0.0, -1,
                 0.0 if k == 0 else 1.0, out, h_k, rows=rows)
            if rows is not None and not last:
                shard.gather(h_full).wait()  # the next round gathers rows of every block
            h_prev = h_k
        if rows is not None:
            shard.pending.append(shard.gather(out_full))
        ctx.graph, ctx.n_gnn, ctx.p, ctx.keys, ctx.pad_row, ctx.sink = graph, n_gnn, p, keys, pad_row, sink
        ctx.E = E
        sink.propagated((graph, n_gnn, p, keys, pad_row, E))
        ctx.mark_non_differentiable(out)
        ctx.set_materialize_grads(False)  # H gets no gradient: no [n, d] zeros for it
        tok = torch.empty((), device=E.device)  # value never read (the dependency is all it carries)
        return out, tok

    @staticmethod
    def backward(ctx, _gH, _gtok):
        sink = ctx.sink
        if sink.ran:  # run eagerly at the last lookup's backward (GradSink.lookup_done)
            return (None,) * 8
        sink.gcn = None
        gE = gcn_backward(sink, ctx.graph, ctx.n_gnn, ctx.p, ctx.keys, ctx.pad_row, ctx.E)
        return gE, None, None, None, None, None, None, None


def gcn_backward(sink, g, n, p, keys, pad_row, E):
    """The GCN backward of one table from its lookup gradient (sink.G): E.grad += Aᵀ-chain(G) + the direct term
    (in place when E.grad exists — returns None — else the gradient is returned)."""
    G = sink.G
    if G is None:
        notify_table(sink.state, E)
        return None
    direct = E.grad is not None
    gE = E.grad if direct else torch.zeros_like(E)
    T = stage_ops()
    work, _, split, _, n_slots, col, val = g.plan(True)
    p = float(p)
    # gE += drop(Aᵀ T_1)/… + G/(n+1) + [i != pad]·G  (rounds before the last: T_{k-1} = G/(n+1) + M_k ⊙ Aᵀ T_k)
    X = T.gcn_backward_rounds(G, work, split, col, val, g.n, n_slots, n, p, flat_keys(keys)) if n > 1 else G
    k0, k1 = keys[0] if n > 0 else (0, 0)
    cuts = row_cuts(sink.state, E) if direct and n > 0 else None
    if cuts is None:
        T.gcn_backward_final(X, G, gE, work, split, col, val, g.n, n_slots, n, p, k0, k1, pad_row, 1.0, 1.0)
    else:  # this table's gradient is final chunk by chunk: its collectives start per chunk (dp.py)
        part = torch.empty(max(n_slots, 1), G.shape[1], device=G.device, dtype=torch.float32)
        for r0, r1 in cuts:
            w0, w1, s0, s1 = g.row_slice(True, r0, r1)
            if w1 > w0:  # roofline accounting of a row-slice launch (bench.py HbmTimer): its rows and edges
                rp = g.host_rowptr(True)
                SPMM_SLICE[work[w0:w1].data_ptr()] = (r1 - r0, int(rp[r1]) - int(rp[r0]))
            T.gcn_backward_final(X, G, gE, work[w0:w1], split[s0:s1], col, val, g.n, n_slots, n, p, k0, k1,
                                 pad_row, 1.0, 1.0, part)
            notify_rows(sink.state, E, r0, r1)
    sink.G = None
    if direct:
        notify_table(sink.state, E)  # E.grad final: its all-reduce runs under the next GCN backward
    return None if direct else gE


class GCNPropFn(Function):
    """``GCN.forward(h, adj)`` at the module API (models/encoders.py:42-48): H = mean(E, A·drop(E), …) as an
    ordinary differentiable op — the gradient of any use of H flows back to E through Aᵀ (same kernels and
    dropout masks as GCNFn, whose fused form serves the training step's embedding lookups instead)."""

    @staticmethod
    def forward(ctx, E, graph, n_gnn, p, keys):
        require_device(E)
        work, _, split, _, n_slots, col, val = graph.plan(False)
        out = stage_ops().gcn_propagate(E.contiguous(), work, split, col, val, graph.n, n_slots, n_gnn, float(p),
                                        flat_keys(keys))
        ctx.graph, ctx.n_gnn, ctx.p, ctx.keys = graph, n_gnn, p, keys
        return out

    @staticmethod
    def backward(ctx, gH):
        G = gH.contiguous()
        n = ctx.n_gnn
        if n == 0:
            return G, None, None, None, None
        T = stage_ops()
        work, _, split, _, n_slots, col, val = ctx.graph.plan(True)
        p = float(ctx.p)
        X = T.gcn_backward_rounds(G, work, split, col, val, ctx.graph.n, n_slots, n, p, flat_keys(ctx.keys)) \
            if n > 1 else G
        gE = torch.empty_like(G)  # the pure gradient: no lookup term, nothing accumulated
        T.gcn_backward_final(X, G, gE, work, split, col, val, ctx.graph.n, n_slots, n, p, ctx.keys[0][0],
                             ctx.keys[0][1], -1, 0.0,
                             0.0)
        return gE, None, None, None, None


# ----------------------------------------------------------------------------- index plans
_side_streams = {}
PLANS_BATCHED = True  # a step's plans in one launch per radix pass (False: one plan at a time, for A/Bs)
PLAN_SRC = {}  # plan buffer data_ptr -> data_ptr of the index tensor it sorts (roofline accounting)


def side_stream(device):
    """The stream the index plans are sorted on (one per device), concurrent with the forward."""
    key = torch.device(device).index
    if key not in _side_streams:
        _side_streams[key] = torch.cuda.Stream(device=device)
    return _side_streams[key]


class IndexPlan:
    """c2dsr_index_plan of one index tensor (stable radix sort into (key, row) order), launched on the
    side stream as soon as the forward sees the indices, so the sort runs under the forward kernels;
    ``get()`` orders the current stream after it and returns the plan buffer."""

    def __init__(self, idx, n_keys, _batch=None):
        if _batch is not None:  # a slice of IndexPlan.many's buffer (launched there)
            self.buf, self.ev = _batch
            return
        nb = int(lib.raw('c2dsr_index_plan_bytes')(idx.numel()))
        buf = torch.empty(nb, dtype=torch.uint8, device=idx.device)
        self.buf, self.ev = IndexPlan._launch([(idx, n_keys)], [buf], [nb], buf)[0]
        if _CHECK_PLANS:
            self.idx, self.n_keys = idx, int(n_keys)

    @staticmethod
    def _launch(pairs, bufs, sizes, whole):
        dev = whole.device
        side = side_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))  # the indices and the buffer are ready
        for (idx, _), buf in zip(pairs, bufs):
            PLAN_SRC[buf.data_ptr()] = idx.data_ptr()
        with torch.cuda.stream(side):  # one stage operator for all the plans, on the side stream
            if PLANS_BATCHED:  # one launch per radix pass over all the plans (c2dsr_index_plans)
                stage_ops().index_plans([idx for idx, _ in pairs], [int(k) for _, k in pairs], whole)
            else:  # plan by plan (the round-5 form; tools/bench_ab.py c2dsr_amd.ops.PLANS_BATCHED)
                for (idx, k), buf, nb in zip(pairs, bufs, sizes):
                    lib('c2dsr_index_plan', idx, idx.numel(), int(k), buf, nb, error_word(), stream())
        whole.record_stream(side)
        ev = torch.cuda.Event()
        ev.record(side)
        return [(buf, ev) for buf in bufs]

    @staticmethod
    def many(pairs):
        """Plans of several (idx, n_keys) in one buffer, one stream hand-off and one event (the host cost of
        a plan is mostly its Python bookkeeping: one training step builds eight)."""
        sizes = [int(lib.raw('c2dsr_index_plan_bytes')(idx.numel())) for idx, _ in pairs]
        whole = torch.empty(sum(sizes), dtype=torch.uint8, device=pairs[0][0].device)  # sizes are 256-aligned
        bufs, o = [], 0
        for nb in sizes:
            bufs.append(whole[o:o + nb])
            o += nb
        out = []
        for (idx, n_keys), be in zip(pairs, IndexPlan._launch(pairs, bufs, sizes, whole)):
            pl = IndexPlan(None, None, _batch=be)
            if _CHECK_PLANS:
                pl.idx, pl.n_keys = idx, int(n_keys)
            out.append(pl)
        return out

    def get(self):
        torch.cuda.current_stream(self.buf.device).wait_event(self.ev)
        if _CHECK_PLANS:
            _check_plan(self.buf, self.idx, self.n_keys)
        return self.buf


_CHECK_PLANS = __import__('os').environ.get('C2DSR_CHECK_PLANS', '0') == '1'
_CHECK_ERR = __import__('os').environ.get('C2DSR_CHECK_ERR', '0') == '1'  # error word only (no sync before use)


def _check_err(ws, off, name):
    err = int(ws[off:off + 4].view(torch.int32).item())
    if err:
        raise HipLibError(f'{name}: inconsistent plan skipped on the device (error word {err:#x})')


def _check_plan(buf, idx, n_keys, seg_ch=16, subp=128):
    """Debug (C2DSR_CHECK_PLANS=1) and tests: the plan against a host restatement (sorted keys, rows, split list,
    the splits' SUBP-piece sub-ranges; csrc/embed.hip plan_layout) before any kernel consumes it.  An index outside
    [0, n_keys) is the key n_keys in the plan (sorted last; csrc/embed.hip prep_keys_kernel)."""
    import numpy as np
    torch.cuda.synchronize()
    b = buf.cpu().numpy()
    x = idx.reshape(-1).cpu().numpy().astype(np.int64)
    n = x.size
    a = lambda v: (v + 255) // 256 * 256  # noqa: E731
    x = np.where((x >= 0) & (x < n_keys), x, n_keys)
    order = np.argsort(x, kind='stable')
    K = x[order]
    o_v = a(4 * n)
    o_sp = o_v + a(4 * n)
    o_ct = o_sp + a(16 * (n // seg_ch + 1))
    o_so = o_ct + a(16)
    o_sb = o_so + a(4 * (n // seg_ch + 2))
    cnt = b[o_ct:o_ct + 16].view(np.int32)
    errs = []
    if not np.array_equal(b[:4 * n].view(np.uint32), K.astype(np.uint32)):
        errs.append('keys')
    if not np.array_equal(b[o_v:o_v + 4 * n].view(np.uint32), order.astype(np.uint32)):
        errs.append('rows')
    ref = []
    for i in range(n):
        if i == 0 or K[i] != K[i - 1]:
            ce = (i // seg_ch + 1) * seg_ch
            if ce < n and K[ce] == K[i]:
                end = int(np.searchsorted(K, K[i], side='right'))
                ref.append((K[i], i // seg_ch, (end - 1) // seg_ch - i // seg_ch + 1, 0))
    ref_so, ref_sb = [], []
    for j, (_, _, span, _) in enumerate(ref):
        ref_so.append(len(ref_sb))
        ref_sb += [(j, y * subp) for y in range(-(-span // subp))]
    ref_so.append(len(ref_sb))
    if int(cnt[1]) != len(ref):
        errs.append(f'splits {int(cnt[1])} != {len(ref)}')
    elif ref:
        got = b[o_sp:o_sp + 16 * len(ref)].view(np.int32).reshape(-1, 4)
        if not np.array_equal(got, np.array(ref, dtype=np.int32).reshape(-1, 4)):
            errs.append('split list')
    if int(cnt[2]) != len(ref_sb):
        errs.append(f'subs {int(cnt[2])} != {len(ref_sb)}')
    else:
        if not np.array_equal(b[o_so:o_so + 4 * len(ref_so)].view(np.int32), np.array(ref_so, dtype=np.int32)):
            errs.append('sub offsets')
        if ref_sb and not np.array_equal(b[o_sb:o_sb + 8 * len(ref_sb)].view(np.int32).reshape(-1, 2),
                                         np.array(ref_sb, dtype=np.int32).reshape(-1, 2)):
            errs.append('sub list')
    if int(cnt[3]) != 0:
        errs.append(f'error word {int(cnt[3]):#x}')
    if errs:
        raise HipLibError(f'index plan mismatch (n={n}, n_keys={n_keys}): {errs}')


def index_plan(state, idx, n_keys):
    """Plan of ``idx`` cached per training step on the StepState (pos tensors are shared by passes)."""
    cache = getattr(state, 'plans', None) if state is not None else None
    if cache is None:
        return IndexPlan(idx, n_keys)
    key = (state.step, idx.data_ptr(), idx.numel(), int(n_keys))
    pl = cache.get(key)
    if pl is None:
        if cache and next(iter(cache))[0] != state.step:
            cache.clear()
        pl = cache[key] = IndexPlan(idx, n_keys)
    return pl


def index_plans(state, pairs):
    """index_plan of every (idx, n_keys) of ``pairs`` (those not cached yet built by one IndexPlan.many)."""
    cache = getattr(state, 'plans', None) if state is not None else None
    if cache is None:
        return IndexPlan.many(pairs)
    if cache and next(iter(cache))[0] != state.step:
        cache.clear()
    todo, keys = [], []
    for idx, n_keys in pairs:
        key = (state.step, idx.data_ptr(), idx.numel(), int(n_keys))
        if key not in cache and key not in keys:
            todo.append((idx, n_keys))
            keys.append(key)
    if todo:
        for key, pl in zip(keys, IndexPlan.many(todo)):
            cache[key] = pl
    return [cache[(state.step, idx.data_ptr(), idx.numel(), int(n_keys))] for idx, n_keys in pairs]


# ----------------------------------------------------------------------------- embedding fuse (K2)
class EmbedFn(Function):
    """x = drop((H[seq] + E[seq])·√d + P[pos])  (models/C2DSR.py:65-71 + encoders.py:30-31)."""

    @staticmethod
    def forward(ctx, tok, E, P, seq, pos, H, scale, p, keys, row_base, sink, pad_row, link=None):
        require_device(E)
        B, L = seq.shape
        d = E.shape[1]
        x = stage_ops().embed_fuse(seq, pos, H, E, None, P, float(scale), float(p), keys[0], keys[1], int(row_base))
        ctx.save_for_backward(seq, pos)
        ctx.scale, ctx.p, ctx.keys, ctx.row_base, ctx.sink, ctx.n_items = scale, p, keys, row_base, sink, E.shape[0]
        ctx.P = P
        ctx.link = link
        ctx.plans = None
        if sink is not None and any(ctx.needs_input_grad):
            sink.lookup_recorded()
        if any(ctx.needs_input_grad[:3]) and (P.requires_grad or sink is not None):  # forward runs under no_grad
            # the sort plans are looked up (or built) when the backward needs them: a trainer enqueues the step's
            # plans where the stream has long kernels queued (trainer.train_batch), not between these launches
            ctx.plans = (sink.state if sink is not None else None, sink is not None, E.shape[0], P.requires_grad,
                         P.shape[0])
        return x

    @staticmethod
    def backward(ctx, gx):
        seq, pos = ctx.saved_tensors
        B, L = seq.shape
        d = gx.shape[-1]
        n = B * L
        G = ctx.sink.buf() if ctx.sink is not None else None
        gP = _grad_target(ctx.P)
        gP_ret = None
        if gP is None and ctx.needs_input_grad[2]:
            gP_ret = torch.zeros_like(ctx.P)
            gP = gP_ret
        if ctx.plans is not None:
            state, on_seq, n_seq, on_pos, n_pos = ctx.plans
            ctx.plans = (index_plan(state, seq, n_seq) if on_seq else None,
                         index_plan(state, pos, n_pos) if on_pos else None)
        parts = ctx.link.take() if ctx.link is not None else None  # gx is a placeholder then (RowsGrad)
        planned = (ctx.plans is not None and (G is None or ctx.plans[0] is not None)
                   and (gP is None or ctx.plans[1] is not None))
        if parts is not None and not planned:
            gx = torch.empty(B, L, d, device=gP.device if gP is not None else G.device, dtype=torch.float32)
            lib('c2dsr_combine_rows', *parts, n, d, gx, stream())
            parts = None
        gx = gx.contiguous() if parts is None else None
        if planned:
            sp = ctx.plans[0].get() if G is not None else None
            pp = ctx.plans[1].get() if gP is not None else None
            # (bench accounting: the rows of the two compact parts, and the index tensor the seq plan sorts)
            if parts is not None:  # the two compact row sources, read through their maps
                stage_ops().embed_fuse_backward(sp, pp, n, d, None, *parts, float(ctx.p), ctx.keys[0], ctx.keys[1],
                                                int(ctx.row_base) * L, float(ctx.scale), G, gP,
                                                [float(parts[0].shape[0] + parts[2].shape[0]), float(seq.data_ptr())])
            else:
                stage_ops().embed_fuse_backward(sp, pp, n, d, gx, None, None, None, None, float(ctx.p), ctx.keys[0],
                                                ctx.keys[1], int(ctx.row_base) * L, float(ctx.scale), G, gP,
                                                [0.0, float(seq.data_ptr())])
            if _CHECK_PLANS or _CHECK_ERR:
                off = int(lib.raw('c2dsr_plan_err_offset')(n))
                for pl in (sp, pp):
                    if pl is not None:
                        _check_err(pl, off, 'c2dsr_embed_bwd_planned')
        else:
            ws_bytes = lib.raw('c2dsr_embed_bwd_workspace')(n, d)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=gx.device)
            lib('c2dsr_embed_bwd', seq, pos, n, d, gx, ctx.keys[0], ctx.keys[1], float(ctx.p), int(ctx.row_base) * L,
                float(ctx.scale), G, ctx.n_items, gP, ctx.P.shape[0], None, ws, ws_bytes, stream())
        return EmbedFn._done(ctx, seq, gP_ret)

    @staticmethod
    def _done(ctx, seq, gP_ret):
        ctx.plans = None
        if WBATCH is not None:  # the last lookup: the deferred weight-gradient products run now
            WBATCH.lookup_done()
        if ctx.sink is not None:
            notify_lookup(ctx.sink.state)
            ctx.sink.lookup_done()
        tok_grad = torch.empty((), device=seq.device)  # value never read (GCNFn.backward reads the sink)
        return tok_grad, None, gP_ret, None, None, None, None, None, None, None, None, None, None


FUSED_PASS = True  # the training step's encoder passes as one stage operator each way (EncoderPassFn)


def fused_pass_ok(precision, B, L, d, n_head):
    """The fused pass covers the step's fast path — d = 256, the row-subset attention, the split-bf16 (fp32 mode, linear1
    guarded) or bf16 projection kernels; any other shape or precision runs op by op (EmbedFn → RowsQKVAttnFn → …)."""
    if not FUSED_PASS or d != 256 or precision not in (FP32, BF16) or not attn_rows_ok(L, d, n_head):
        return False
    M = B * L  # the compact row counts are at most B·L (the support checks bound sizes from above)
    kind = 'x3' if precision == FP32 else 'b16'
    ok = all(rg_kind(precision, M, n, k) == kind for n, k in ((d, d), (2 * d, d), (d, 2 * d)))
    ok = ok and all(wg_kind(precision, M, n, d) == kind for n in (d, 2 * d))
    return ok and (precision == BF16 or (RELU_GUARD and relu_guard_ok(M, d, d)))


class EncoderPassFn(Function):
    """One training pass (models/C2DSR.py:64-85 → encoders.py:29-33, TransformerEncoder with one post-norm layer + the
    final LayerNorm) as ONE stage operator each way: c2dsr::encoder_pass / encoder_pass_backward
    (csrc_torch/encoder_ops.cpp).  The same kernels in the same order as the op-by-op path EmbedFn → RowsQKVAttnFn →
    LinearFn → AddLNFn → LinearFn ×2 → AddLN2Fn (bit-identical results): the embedding fuse, Q at the rows the loss
    reads (rs) and K / V at the padding rows (ks), the row-wise rest of the layer on the rs rows.  Returns the [n, d]
    output rows (the loss head reads them through rs.inv).  Backward: the weight-gradient operands go to the step's
    WGradBatch (grouped per weight across passes) and the input gradient, in its two compact parts, straight into
    the embedding's deterministic segment sums (G: the GCN output's gradient sink; the position table)."""

    @staticmethod
    def forward(ctx, tok, E, P, seq, pos, H, att, nm, rs, ks, keys, p, row_off, precision, sink, scale):
        require_device(E)
        lay = att.encoder.layers[0]
        at = lay.self_attn
        d = E.shape[1]
        kind = 'x3' if precision == FP32 else 'b16'
        w = [at.in_proj_weight, at.in_proj_bias, at.out_proj.weight, at.out_proj.bias, lay.linear1.weight,
             lay.linear1.bias, lay.linear2.weight, lay.linear2.bias, lay.norm1.weight, lay.norm1.bias, lay.norm2.weight,
             lay.norm2.bias, nm.weight, nm.bias]
        wd = [t.detach() for t in w]
        Wq, Wkv = wd[0][:d], wd[0][d:]
        img = [weight_img(Wq, kind), weight_img(Wkv, kind), weight_img(wd[2], kind), weight_img(wd[4], kind),
               weight_img(wd[6], kind)]
        gws = None
        if precision == FP32:
            img.append(WEIGHTS.get(wd[4], False, layout='norm2'))
            nq = rs.n
            wsb = int(lib.raw('c2dsr_rgemm_guard_workspace')(max(nq, 1), d))
            gws = _GUARD_WS.get(E.device)
            if gws is None or gws.numel() < wsb:  # zeroed once: every call leaves its flags cleared
                gws = _GUARD_WS[E.device] = torch.zeros(max(wsb, 1 << 20), device=E.device, dtype=torch.uint8)
        else:
            img.append(torch.empty(0, device=E.device))
        rsi, ksi = rs.idx[:rs.n], ks.idx[:ks.n]
        outs = stage_ops().encoder_pass(seq, pos, H, E, P, float(scale), wd, img, rsi, rs.off, ksi, ks.off,
                                        int(att.idx_pad), int(att.n_head), float(p), flat_keys(keys),
                                        [float(lay.norm1.eps), float(lay.norm2.eps), float(nm.eps)], int(row_off),
                                        0 if precision == FP32 else 1, gws)
        ctx.saved = outs[1:]
        ctx.args = (seq, pos, w, wd, rs, ks, rsi, ksi, keys, p, row_off, precision, att, scale)
        ctx.sink, ctx.P, ctx.n_items = sink, P, E.shape[0]
        if sink is not None and any(ctx.needs_input_grad):
            sink.lookup_recorded()
        return outs[0]

    @staticmethod
    def backward(ctx, gout):
        seq, pos, w, wd, rs, ks, rsi, ksi, keys, p, row_off, precision, att, scale = ctx.args
        d = wd[2].shape[0]
        kind = 'x3' if precision == FP32 else 'b16'
        imgT = [weight_img(wd[0][:d], kind, True), weight_img(wd[0][d:], kind, True), weight_img(wd[2], kind, True),
                weight_img(wd[4], kind, True), weight_img(wd[6], kind, True)]
        sink = ctx.sink
        G = sink.buf() if sink is not None else None
        gP = _grad_target(ctx.P)
        gP_ret = None
        if gP is None and ctx.needs_input_grad[2]:
            gP_ret = gP = torch.zeros_like(ctx.P)
        state = sink.state if sink is not None else None
        sp = index_plan(state, seq, ctx.n_items).get() if G is not None else None
        pp = index_plan(state, pos, ctx.P.shape[0]).get() if gP is not None else None
        lng = []
        for t in w[8:]:
            g = _grad_target(t)
            lng.append(g if g is not None else torch.zeros_like(t))  # a frozen LayerNorm parameter: scratch
        pairs = stage_ops().encoder_pass_backward(gout.contiguous(), ctx.saved, seq, wd, imgT, rsi, rs.inv, rs.off, ksi,
                                                  ks.inv, ks.off, int(att.idx_pad), int(att.n_head), float(p),
                                                  flat_keys(keys), int(row_off), 0 if precision == FP32 else 1, lng,
                                                  sp, pp, float(scale), G, gP)
        ctx.saved = None
        # weight / bias gradients of linear2, linear1, out_proj, in_proj (q rows, k/v rows) — the op-by-op path's order
        gWin, gbin = _grad_target(w[0]), _grad_target(w[1])
        targets = [(_grad_target(w[6]), _grad_target(w[7])), (_grad_target(w[4]), _grad_target(w[5])),
                   (_grad_target(w[2]), _grad_target(w[3])),
                   (None if gWin is None else gWin[:d], None if gbin is None else gbin[:d]),
                   (None if gWin is None else gWin[d:], None if gbin is None else gbin[d:])]
        for (gW, gb), dY, X in zip(targets, pairs[0::2], pairs[1::2]):
            if gW is None or X.shape[0] == 0:
                continue
            wgemm(dY, X, gW, T=X.shape[0], N=gW.shape[0], D=X.shape[1], db=gb, x3=precision == FP32)
        if WBATCH is not None:  # this pass's lookup is done (the last one flushes the deferred products)
            WBATCH.lookup_done()
        if sink is not None:
            notify_lookup(sink.state)
            sink.lookup_done()
        tok_grad = torch.empty((), device=gout.device)
        return (tok_grad, None, gP_ret) + (None,) * 13


class RowsGrad:
    """Hands the row-subset attention layer's input gradient to the embedding backward as its two compact
    parts (query rows, key rows; RowsQKVAttnFn) when that layer reads the embedding output directly (one
    encoder layer): the embedding's segment sums read the parts through their row maps
    (c2dsr_embed_bwd_planned_rows) and the [B, L, d] gradient is never written.  Autograd carries a
    zero-stride placeholder of the right shape between the two nodes; the link is the only consumer path,
    so nothing else reads the placeholder."""

    def __init__(self):
        self.parts = None

    def take(self):
        parts, self.parts = self.parts, None
        return parts


class PosDropFn(Function):
    """x = drop(seq_enc + P[pos])  — SelfAttention.forward on a caller-provided seq_enc (encoders.py:30-31)."""

    @staticmethod
    def forward(ctx, xin, P, pos, p, keys, row_base):
        B, L, d = xin.shape
        x = torch.empty_like(xin)
        lib('c2dsr_embed_fwd', pos, pos, B * L, d, None, None, xin, P, 1.0, keys[0], keys[1], float(p),
            int(row_base) * L, x, 0, P.shape[0], error_word(), stream())
        ctx.save_for_backward(pos)
        ctx.p, ctx.keys, ctx.row_base, ctx.P = p, keys, row_base, P
        return x

    @staticmethod
    def backward(ctx, gx):
        (pos,) = ctx.saved_tensors
        B, L = pos.shape
        gx = gx.contiguous()
        d = gx.shape[-1]
        n = B * L
        gP = _grad_target(ctx.P)
        gP_ret = None
        if gP is None and ctx.needs_input_grad[1]:
            gP_ret = torch.zeros_like(ctx.P)
            gP = gP_ret
        gxin = torch.empty_like(gx)
        ws_bytes = lib.raw('c2dsr_embed_bwd_workspace')(n, d)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=gx.device)
        lib('c2dsr_embed_bwd', pos, pos, n, d, gx, ctx.keys[0], ctx.keys[1], float(ctx.p), int(ctx.row_base) * L,
            1.0, None, 0, gP, ctx.P.shape[0], gxin, ws, ws_bytes, stream())
        return gxin, gP_ret, None, None, None, None


class PosAddFn(Function):
    """``seq_enc += self.pos_emb(pos)`` IN PLACE (encoders.py:30, Q20): the caller's tensor is mutated as the
    reference's in-place add mutates it (c2dsr_embed_fwd with Xin = X), and autograd sees an in-place op
    (mark_dirty): the gradient of the mutated tensor flows to the original values and, summed by position,
    to the position table."""

    @staticmethod
    def forward(ctx, xin, P, pos):
        require_device(xin)
        B, L, d = xin.shape
        lib('c2dsr_embed_fwd', pos, pos, B * L, d, None, None, xin, P, 1.0, 0, 0, 0.0, 0, xin, 0, P.shape[0],
            error_word(), stream())
        ctx.mark_dirty(xin)
        ctx.save_for_backward(pos)
        ctx.P = P
        return xin

    @staticmethod
    def backward(ctx, gx):
        (pos,) = ctx.saved_tensors
        gx = gx.contiguous()
        B, L = pos.shape
        d = gx.shape[-1]
        n = B * L
        gP = _grad_target(ctx.P)
        gP_ret = None
        if gP is None and ctx.needs_input_grad[1]:
            gP_ret = torch.zeros_like(ctx.P)
            gP = gP_ret
        if gP is None:
            return gx, None, None
        gxin = torch.empty_like(gx)
        ws_bytes = lib.raw('c2dsr_embed_bwd_workspace')(n, d)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=gx.device)
        lib('c2dsr_embed_bwd', pos, pos, n, d, gx, 0, 0, 0.0, 0, 1.0, None, 0, gP, ctx.P.shape[0], gxin, ws, ws_bytes,
            stream())
        return gxin, gP_ret, None


class DropFn(Function):
    """y = dropout(x) with the stateless hash masks (encoders.py:31), index (row_base + row)·d + col."""

    @staticmethod
    def forward(ctx, x, p, keys, row_base):
        y = torch.empty_like(x)
        lib('c2dsr_add_dropout', None, x.contiguous(), x.numel(), x.shape[-1], keys[0], keys[1], float(p),
            int(row_base), y, stream())
        ctx.p, ctx.keys, ctx.row_base = p, keys, row_base
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        lib('c2dsr_add_dropout', None, dy, dy.numel(), dy.shape[-1], ctx.keys[0], ctx.keys[1], float(ctx.p),
            int(ctx.row_base), dx, stream())
        return dx, None, None, None


# ----------------------------------------------------------------------------- attention
class AttnFn(Function):
    """SDPA core with causal + inverted key-padding mask (Q1, Q2)."""

    @staticmethod
    def forward(ctx, qkv, seq, pad, n_head, p, keys, b_base):
        B, L, d3 = qkv.shape
        d = d3 // 3
        out = torch.empty(B, L, d, device=qkv.device, dtype=torch.float32)
        P = torch.empty(int(lib.raw('c2dsr_attn_psave_floats')(B, L, d, n_head)), device=qkv.device,
                        dtype=torch.float32)  # the kernels' own layout
        lib('c2dsr_attn_fwd', qkv, seq, int(pad), B, L, d, n_head, keys[0], keys[1], float(p), int(b_base), out, P,
            stream())
        ctx.save_for_backward(qkv, seq, P)
        ctx.pad, ctx.n_head, ctx.p, ctx.keys, ctx.b_base = pad, n_head, p, keys, b_base
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, seq, P = ctx.saved_tensors
        B, L, d3 = qkv.shape
        d = d3 // 3
        dqkv = torch.empty_like(qkv)
        lib('c2dsr_attn_bwd', qkv, seq, int(ctx.pad), B, L, d, ctx.n_head, ctx.keys[0], ctx.keys[1], float(ctx.p),
            int(ctx.b_base), P, dout.contiguous(), dqkv, stream())
        return dqkv, None, None, None, None, None, None


class QKVAttnFn(Function):
    """qkv = x·W_inᵀ + b_in, then the attention core (models/encoders.py:33 → MultiheadAttention: in_proj and
    SDPA) as one autograd node, so that in bf16 mode the attention backward can hand dqkv to the in_proj
    backward GEMMs in bf16 (c2dsr_attn_bwd_b16 → c2dsr_rgemm_aux_b16a / c2dsr_wgemm_b16y): their only
    consumers read it as a bf16 MFMA operand, so the values are the ones they would round to, at half the
    bytes.  Otherwise identical to LinearFn followed by AttnFn.  res: the ResidualLink of the layer input."""

    @staticmethod
    def forward(ctx, x, W, b, seq, pad, n_head, p, keys, b_base, precision, res=None):
        require_device(x)
        N, K = W.shape
        M = x.numel() // K
        qkv = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
        kind = rg_kind(precision, M, N, K)
        if kind:
            rgemm(x, weight_img(W, kind), qkv, M=M, N=N, K=K, bias=b, x3=kind == 'x3', frag=True)
        else:
            gemm(x, W, qkv, M=M, N=N, K=K, transB=1, bias=b, precision=precision)
        B, L, d3 = qkv.shape
        d = d3 // 3
        out = torch.empty(B, L, d, device=x.device, dtype=torch.float32)
        P = torch.empty(int(lib.raw('c2dsr_attn_psave_floats')(B, L, d, n_head)), device=x.device,
                        dtype=torch.float32)
        lib('c2dsr_attn_fwd', qkv, seq, int(pad), B, L, d, n_head, keys[0], keys[1], float(p), int(b_base), out, P,
            stream())
        ctx.save_for_backward(x, W, qkv, seq, P)
        ctx.pad, ctx.n_head, ctx.p, ctx.keys, ctx.b_base = pad, n_head, p, keys, b_base
        ctx.b, ctx.precision, ctx.relu_p, ctx.res, ctx.ff, ctx.ff_role = b, precision, None, res, None, None
        return out

    @staticmethod
    def backward(ctx, dout):
        x, W, qkv, seq, P = ctx.saved_tensors
        B, L, d3 = qkv.shape
        d = d3 // 3
        M = B * L
        s = stream()
        b16 = (ctx.precision == BF16 and bool(lib.raw('c2dsr_attn_bwd_b16_supported')(L, d, ctx.n_head))
               and rgemm_ok(M, d, d3) and wgemm_ok(M, d3, d))
        args = (qkv, seq, int(ctx.pad), B, L, d, ctx.n_head, ctx.keys[0], ctx.keys[1], float(ctx.p), int(ctx.b_base), P,
                dout.contiguous())
        if b16:
            dqkv = torch.empty(qkv.shape, device=qkv.device, dtype=torch.bfloat16)
            lib('c2dsr_attn_bwd_b16', *args, dqkv, s)
        else:
            dqkv = torch.empty_like(qkv)
            lib('c2dsr_attn_bwd', *args, dqkv, s)
        dx = linear_backward(ctx, x, W, None, dqkv, ctx.needs_input_grad[0])
        return (dx,) + (None,) * 10




def attn_rows_ok(L, d, n_head):
    return bool(lib.raw('c2dsr_attn_rows_supported')(L, d, n_head))


def _proj(x, W, b, y, precision):
    """y = x·Wᵀ + b (x fp32 [M, K], W a row range of a projection weight)."""
    N, K = W.shape
    M = x.shape[0]
    if M == 0:
        return y
    kind = rg_kind(precision, M, N, K)
    if kind:
        rgemm(x, weight_img(W, kind), y, M=M, N=N, K=K, bias=b, x3=kind == 'x3', frag=True)
    else:
        gemm(x, W, y, M=M, N=N, K=K, transB=1, bias=b, precision=precision)
    return y


def _proj_backward(x, W, dy, dx, acc, gW, gb, precision):
    """dx (+)= dy·W  (acc: dx holds a gradient to add to) and gW += dyᵀ·x, gb += Σ dy for y = x·Wᵀ + b over a
    row range of the weight; dy fp32 or bf16 (then every product takes the bf16-operand kernels)."""
    N, K = W.shape
    M = x.shape[0]
    if M == 0:
        return
    kind = rg_kind(precision, M, K, N)
    if kind:
        rgemm(dy, weight_img(W, kind, trans=True), dx, M=M, N=K, K=N, aux_mode=AUX_ACC if acc else 0,
              aux=dx if acc else None, x3=kind == 'x3', frag=True)
    else:
        gemm(dy, W, dx, M=M, N=K, K=N, beta=1.0 if acc else 0.0, precision=precision)
    wk = wg_kind(precision, M, N, K)
    if gW is not None and wk:
        wgemm(dy, x, gW, T=M, N=N, D=K, db=gb, x3=wk == 'x3')
    else:
        if gW is not None:
            gemm(dy, x, gW, M=N, N=K, K=M, transA=1, lda=N, ldb=K, beta=1.0, precision=precision)
        if gb is not None:
            colsum(dy, M, N, N, gb)


class RowsQKVAttnFn(Function):
    """The in_proj + attention core of the LAST post-norm encoder layer of a training pass, on the rows that
    matter only (models/encoders.py:33 → MultiheadAttention; everything after the attention is row-wise and
    the loss reads the rows of ``rs``): Q is projected for the query rows rs (from xc = x[rs], the rows the
    layer's residual reads too), K / V for the padding rows ks — the only keys any query may attend to (Q1) —
    and the attention runs on those compact rows (c2dsr_attn_fwd_rows).  Returns the [n_q, d] attention
    output of the rs rows, equal to the full layer's at those rows up to the order of the key sums.
    Backward: dq, dkv (bf16 in bf16 mode, as QKVAttnFn) → dx = dq·Wq (+ the parked LN gradient of the rs rows,
    ResidualLink) on the query rows + dkv·Wkv on the key rows, combined into the [B, L, d] input gradient
    (rows in neither set get 0: nothing downstream reads them)."""

    @staticmethod
    def forward(ctx, x, xc, W, b, seq, pad, n_head, p, keys, b_base, precision, rs, ks, res=None, link=None):
        require_device(x)
        B, L, d = x.shape
        if not attn_rows_ok(L, d, n_head) or rs.off is None or ks.off is None:
            raise HipLibError('RowsQKVAttnFn: unsupported shape or row sets without per-sequence offsets')
        nq, nk = rs.n, ks.n
        xk = torch.empty(nk, d, device=x.device, dtype=torch.float32)
        if nk:
            lib('c2dsr_gather_rows', x.detach(), d, ks.idx, nk, d, xk, stream())
        q = _proj(xc, W[:d], b[:d], torch.empty(nq, d, device=x.device, dtype=torch.float32), precision)
        kv = _proj(xk, W[d:], b[d:], torch.empty(nk, 2 * d, device=x.device, dtype=torch.float32), precision)
        out = torch.empty(nq, d, device=x.device, dtype=torch.float32)
        P = torch.empty(int(lib.raw('c2dsr_attn_psave_floats')(B, L, d, n_head)), device=x.device,
                        dtype=torch.float32)
        lib('c2dsr_attn_fwd_rows', q, kv, seq, int(pad), rs.idx, rs.off, ks.idx, ks.off, B, L, d, n_head, keys[0],
            keys[1], float(p), int(b_base), out, P, stream())
        ctx.save_for_backward(xc, xk, W, q, kv, seq, P)
        ctx.b, ctx.pad, ctx.n_head, ctx.p, ctx.keys, ctx.b_base = b, pad, n_head, p, keys, b_base
        ctx.precision, ctx.rs, ctx.ks, ctx.res, ctx.shape, ctx.link = precision, rs, ks, res, (B, L, d), link
        return out

    @staticmethod
    def backward(ctx, dout):
        xc, xk, W, q, kv, seq, P = ctx.saved_tensors
        B, L, d = ctx.shape
        rs, ks = ctx.rs, ctx.ks
        nq, nk = q.shape[0], kv.shape[0]
        s = stream()
        b16 = (ctx.precision == BF16 and rgemm_ok(max(nq, 1), d, d) and rgemm_ok(max(nk, 1), d, 2 * d)
               and wgemm_ok(max(nq, 1), d, d) and wgemm_ok(max(nk, 1), 2 * d, d))
        gt = torch.bfloat16 if b16 else torch.float32
        dq = torch.empty(nq, d, device=q.device, dtype=gt)
        dkv = torch.empty(nk, 2 * d, device=q.device, dtype=gt)
        lib('c2dsr_attn_bwd_rows', q, kv, seq, int(ctx.pad), rs.idx, rs.off, ks.idx, ks.off, B, L, d, ctx.n_head,
            ctx.keys[0], ctx.keys[1], float(ctx.p), int(ctx.b_base), P, dout.contiguous(), dq, dkv, int(b16), s)
        park = None
        if ctx.res is not None:
            park, ctx.res.grad = ctx.res.grad, None
        gW, gb = _grad_target(W), _grad_target(ctx.b)
        dxq = park if park is not None else torch.empty(nq, d, device=q.device, dtype=torch.float32)
        _proj_backward(xc, W[:d], dq, dxq, park is not None, None if gW is None else gW[:d],
                       None if gb is None else gb[:d], ctx.precision)
        dxk = torch.empty(nk, d, device=q.device, dtype=torch.float32)
        _proj_backward(xk, W[d:], dkv, dxk, False, None if gW is None else gW[d:], None if gb is None else gb[d:],
                       ctx.precision)
        dx = None
        if ctx.needs_input_grad[0] and ctx.link is not None:  # the embedding backward reads the parts (RowsGrad)
            ctx.link.parts = (dxq, rs.inv, dxk, ks.inv)
            dx = torch.empty(1, 1, 1, device=q.device).expand(B, L, d)
        elif ctx.needs_input_grad[0]:
            dx = torch.empty(B, L, d, device=q.device, dtype=torch.float32)
            lib('c2dsr_combine_rows', dxq, rs.inv, dxk, ks.inv, B * L, d, dx, s)
        return (dx,) + (None,) * 14


# ----------------------------------------------------------------------------- residual / layernorm
class AddLNFn(Function):
    """y = LayerNorm(a + drop(b))  (b may be None: plain LayerNorm of a); eps 1e-8."""

    @staticmethod
    def forward(ctx, a, b, w, bias, p, keys, row_base, eps, res=None, rowmap=None):
        d = a.shape[-1]
        rows = a.numel() // d
        y = torch.empty_like(a)
        xsave = torch.empty_like(a) if b is not None else None
        mean = torch.empty(rows, device=a.device)
        rstd = torch.empty(rows, device=a.device)
        lib('c2dsr_add_ln_fwd', a, b, rows, d, keys[0], keys[1], float(p), int(row_base), rowmap, w, bias, float(eps),
            xsave, y, mean, rstd, stream())
        ctx.save_for_backward(xsave if b is not None else a, mean, rstd)
        ctx.w, ctx.bias, ctx.p, ctx.keys, ctx.row_base, ctx.has_b = w, bias, p, keys, row_base, b is not None
        ctx.res = res
        ctx.rowmap = rowmap
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        d = x.shape[-1]
        rows = x.numel() // d
        dy = dy.contiguous()
        da = torch.empty_like(x)
        db = torch.empty_like(x) if ctx.has_b else None
        gw, gb = _grad_target(ctx.w), _grad_target(ctx.bias)
        ws = torch.empty(lib.raw('c2dsr_ln_bwd_workspace')(d), dtype=torch.uint8, device=x.device)
        lib('c2dsr_ln_bwd', x, mean, rstd, ctx.w, dy, rows, d, da, 0, db, ctx.keys[0], ctx.keys[1], float(ctx.p),
            int(ctx.row_base), ctx.rowmap, gw, gb, ws, stream())
        if ctx.res is not None:  # parked for the layer's first projection (ResidualLink)
            ctx.res.grad = da
            da = None
        return da, db, None, None, None, None, None, None, None, None


class AddLN2Fn(Function):
    """y = LN_F(LN_2(a + drop(b))·w2 + b2)·wF + bF — the last post-norm layer's norm2 and the encoder's final
    norm (models/encoders.py:23-27 → transformer.py, Q16) in one pass each way (c2dsr_add_ln2_fwd / _ln2_bwd):
    the intermediate row is neither written nor re-read.  res: the ResidualLink of a (its gradient is parked
    there for linear1's dX product); rowmap: dropout rows of a row subset (as AddLNFn)."""

    @staticmethod
    def forward(ctx, a, b, w2, b2, wF, bF, p, keys, row_base, eps2, epsF, res=None, rowmap=None):
        d = a.shape[-1]
        rows = a.numel() // d
        y = torch.empty_like(a)
        xsave = torch.empty_like(a)
        st = torch.empty(4, rows, device=a.device)
        lib('c2dsr_add_ln2_fwd', a, b.contiguous(), rows, d, keys[0], keys[1], float(p), int(row_base), rowmap, w2,
            b2, float(eps2), wF, bF, float(epsF), xsave, y, st, stream())
        ctx.save_for_backward(xsave, st)
        ctx.ws, ctx.p, ctx.keys, ctx.row_base, ctx.res, ctx.rowmap = (w2, b2, wF, bF), p, keys, row_base, res, rowmap
        return y

    @staticmethod
    def backward(ctx, dy):
        xsave, st = ctx.saved_tensors
        d = xsave.shape[-1]
        rows = xsave.numel() // d
        w2, b2, wF, bF = ctx.ws
        da = torch.empty_like(xsave)
        db = torch.empty_like(xsave)
        ws = torch.empty(lib.raw('c2dsr_ln2_bwd_workspace')(d), dtype=torch.uint8, device=xsave.device)
        lib('c2dsr_ln2_bwd', xsave, st, w2, b2, wF, dy.contiguous(), rows, d, da, db, ctx.keys[0], ctx.keys[1],
            float(ctx.p), int(ctx.row_base), ctx.rowmap, _grad_target(w2), _grad_target(b2), _grad_target(wF),
            _grad_target(bF), ws, stream())
        if ctx.res is not None:  # parked for linear1's dX product (ResidualLink)
            ctx.res.grad = da
            da = None
        return (da, db) + (None,) * 11


class AddDropFn(Function):
    """y = a + drop(b)  (pre-norm residual)."""

    @staticmethod
    def forward(ctx, a, b, p, keys, row_base):
        d = a.shape[-1]
        y = torch.empty_like(a)
        lib('c2dsr_add_dropout', a, b.contiguous(), a.numel(), d, keys[0], keys[1], float(p), int(row_base), y,
            stream())
        ctx.p, ctx.keys, ctx.row_base = p, keys, row_base
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        db = torch.empty_like(dy)
        lib('c2dsr_add_dropout', None, dy, dy.numel(), dy.shape[-1], ctx.keys[0], ctx.keys[1], float(ctx.p),
            int(ctx.row_base), db, stream())
        return dy, db, None, None, None


# ----------------------------------------------------------------------------- bilinear (D_a / D_b)
class BilinearFn(Function):
    """nn.Bilinear(d, d, 1): s = x1ᵀ W x2 (+b)  (models/C2DSR.py:46-55 used at trainer.py:104-108)."""

    @staticmethod
    def forward(ctx, x1, x2, W, b):
        B, d = x1.shape
        U = torch.empty(B, d, device=x1.device, dtype=torch.float32)
        gemm(x2, W, U, M=B, N=d, K=d, transB=1)
        out = torch.empty(B, 1, device=x1.device, dtype=torch.float32)
        lib('c2dsr_rowdot', x1, d, U, d, B, d, b, out, 1, stream())
        ctx.save_for_backward(x1, x2, U)
        ctx.W, ctx.b = W, b
        return out

    @staticmethod
    def backward(ctx, dout):
        x1, x2, U = ctx.saved_tensors
        B, d = x1.shape
        ds = dout.contiguous().reshape(B)
        s = stream()
        dx1 = torch.empty_like(x1)
        lib('c2dsr_rowscale', U, ds, B * d, d, dx1, 0, s)
        dU = torch.empty_like(x1)
        lib('c2dsr_rowscale', x1, ds, B * d, d, dU, 0, s)
        dx2 = torch.empty_like(x2)
        gemm(dU, ctx.W, dx2, M=B, N=d, K=d)
        gW = _grad_target(ctx.W)
        if gW is not None:
            gemm(dU, x2, gW, M=d, N=d, K=B, transA=1, beta=1.0)
        gb = _grad_target(ctx.b)
        if gb is not None:
            colsum(ds, B, 1, 1, gb)
        return dx1, dx2, None, None


# ----------------------------------------------------------------------------- evaluation (§8 f1)
def eval_rank(h_share, h_a, h_b, idx_last_a, idx_last_b, xory, gt, neg, Wa, ba, Wb, bb):
    """rank[i] = 1 + #(s(neg) > s(gt)) with s = classifier_dom(h_share[i,-1] + h_dom[i, idx_last_dom[i]])
    (trainer.py:162-181), all rows at once (csrc/eval.hip).  Returns int32 [B] on the device."""
    require_device(h_share)
    B, L, d = h_share.shape
    for t in (h_a, h_b):
        if t.shape != h_share.shape:
            raise ValueError('h_share / hx / hy shapes differ')
    n_neg = neg.shape[1] if neg.dim() == 2 else 0
    ints = [x.reshape(-1).contiguous().long() for x in (idx_last_a, idx_last_b, xory, gt)]
    for x in ints:
        if x.numel() != B:
            raise ValueError('idx_last / xory / gt must hold one entry per row')
    neg = neg.contiguous().long()
    rank = torch.empty(B, dtype=torch.int32, device=h_share.device)
    lib('c2dsr_eval_rank', h_share.contiguous(), h_a.contiguous(), h_b.contiguous(), B, L, d, *ints, neg, n_neg,
        Wa.contiguous(), ba.contiguous(), Wa.shape[0], Wb.contiguous(), bb.contiguous(), Wb.shape[0], rank, stream())
    return rank


def rank_metrics(rank, xory, dom, sums):
    """sums[0..7] += (hr5, hr20, mrr5, mrr20, ndcg5, ndcg20, count, n_bad) of the rows of domain ``dom``
    (utils/metrics.py:4-19, fp64 on the device)."""
    require_device(rank)
    xory = xory.reshape(-1).contiguous().long()
    lib('c2dsr_rank_metrics', rank, xory, rank.numel(), int(dom), sums, stream())
    return sums
