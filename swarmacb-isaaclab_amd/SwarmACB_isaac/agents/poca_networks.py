"""MA-POCA actor / critic networks (drop-in for agents/poca_networks.py).

The module tree, parameter names and initialisation order follow the
reference (poca_networks.py:58-882), so its state_dicts and checkpoints load
into these classes unchanged and a seeded construction draws the same weights.

What is MI355X-specific is the critic's rollout-time evaluation: under
``torch.no_grad()`` on the GPU (how all three trainers call ``critic_pass``,
``joint_action_pass``, ``baseline`` and ``all_baselines`` once per decision),
the residual self-attention runs as the fused HIP kernel of
include/swarmcritic.h. The entity rows of an env are embedded, normalised and
projected once (2N rows instead of the reference's N x N set rows), the
kernel forms every counterfactual set itself and runs fc_out on the matrix
cores. With autograd enabled (the PPO update) the PyTorch path below runs;
it restates the reference math operation by operation.
"""

from __future__ import annotations

import contextlib
import ctypes as C
import math
import os

import torch
import torch.nn as nn
from torch.distributions import Normal

from .. import _native

Swish = nn.SiLU  # ML-Agents' Swish

_KERNEL_INITS = {
    "kaiming_normal": lambda w: nn.init.kaiming_normal_(w, nonlinearity="linear"),
    "normal": nn.init.normal_,
    "xavier_uniform": nn.init.xavier_uniform_,
}


# rows from which a layer's weight gradient is split over row chunks (A/B: profiles/r04/train/splitk_rows_ab.txt)
SPLITK_MIN_ROWS = int(os.environ.get("SWARM_SPLITK_MIN_ROWS", "4096"))
SPLITK_CHUNK_ROWS = int(os.environ.get("SWARM_SPLITK_CHUNK_ROWS", "1024"))   # rows per chunk of that split
# rows per chunk when the layer's input or output is at most 16 wide (the entity embeddings' 5 / 11
# inputs, a value head's 1 output): each chunk's product is one small tile, so shorter chunks give
# the batched GEMM more tiles for the same work (0: SPLITK_CHUNK_ROWS for every layer)
SPLITK_NARROW_ROWS = int(os.environ.get("SWARM_SPLITK_NARROW_ROWS", "0"))
SPLITK_SLAB_ROWS = 256     # rows per column-sum slab of its bias gradient
# False (or SWARM_SPLITK_SUMS=0): the chunk / bias sums run torch's reductions
SPLITK_NATIVE_SUMS = os.environ.get("SWARM_SPLITK_SUMS", "1") != "0"


class _SplitKLinear(torch.autograd.Function):
    """y = x W^T + b whose weight gradient dW = dy^T x sums over R >= SPLITK_MIN_ROWS
    rows (the critic's entity rows: every env x agent x entity of a minibatch). As one
    GEMM that is an (out x in) output with a 40k-deep reduction: a dozen output tiles,
    i.e. a dozen busy CUs of 256. Split into R / SPLITK_CHUNK_ROWS row chunks it is one
    batched GEMM with hundreds of tiles plus a sum over the chunks (fp32 sums in another
    order; the forward and dx are the plain GEMMs)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return torch.addmm(bias, x, weight.t()) if bias is not None else x.mm(weight.t())

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dy.mm(weight) if ctx.needs_input_grad[0] else None
        dw, db = _split_rows_weight_grad(dy, x, ctx.has_bias)
        return dx, dw, db


def _split_rows_weight_grad(dy, x, has_bias: bool):
    """(dy^T x, column sums of dy or None) over R >= SPLITK_CHUNK_ROWS rows as _SplitKLinear
    computes its weight gradient: one batched GEMM over row chunks, then the chunk sums."""
    R = x.shape[0]
    out_f = dy.shape[1]
    chunk = SPLITK_CHUNK_ROWS
    if SPLITK_NARROW_ROWS > 0 and min(x.shape[1], out_f) <= 16:
        chunk = SPLITK_NARROW_ROWS
    c = R // chunk
    L = R // c
    main = c * L
    dyc = dy[:main].view(c, L, out_f)
    parts = torch.bmm(dyc.transpose(1, 2), x[:main].view(c, L, x.shape[1]))
    if SPLITK_NATIVE_SUMS and dy.is_cuda and out_f % 4 == 0 and out_f <= 1024:
        # the chunk sum of the partial products and the bias gradient (column sums of dy
        # per slab, then over the slabs) in two launches (swarm_splitk_colsum / _finish)
        dy = dy.contiguous()
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(dy.device).cuda_stream)
        dw = torch.empty(out_f, x.shape[1], dtype=dy.dtype, device=dy.device)
        db, pb, slabs = None, None, 0
        if has_bias:
            slabs = (R + SPLITK_SLAB_ROWS - 1) // SPLITK_SLAB_ROWS
            pb = torch.empty(slabs, out_f, dtype=dy.dtype, device=dy.device)
            db = torch.empty(out_f, dtype=dy.dtype, device=dy.device)
            _native.check(lib.swarm_splitk_colsum(R, out_f, SPLITK_SLAB_ROWS, _ptr(dy), _ptr(pb), stream),
                          "swarm_splitk_colsum")
        _native.check(lib.swarm_splitk_finish(c, dw.numel(), _ptr(parts), _ptr(dw), slabs,
                                              out_f if has_bias else 0, _ptr(pb), _ptr(db), stream),
                      "swarm_splitk_finish")
        if main < R:
            dw.addmm_(dy[main:].t(), x[main:])
        return dw, db
    dw = parts.sum(dim=0)
    db = dyc.sum(dim=1).sum(dim=0) if has_bias else None
    if main < R:
        dw.addmm_(dy[main:].t(), x[main:])
        if db is not None:
            db += dy[main:].sum(dim=0)
    return dw, db


# Layers over [WGRAD_MIN_ROWS, SPLITK_MIN_ROWS) rows (the update's 2,048-row minibatch MLPs and LSTM
# inputs) take their weight and bias gradients from ONE swarm_wgrad launch instead of the library's
# (out x in) GEMM with a 2,048-deep reduction (14-28 us each at C5) plus a column-sum kernel.
WGRAD_MIN_ROWS = 128
WGRAD_NATIVE = os.environ.get("SWARM_WGRAD", "1") != "0"


def _wgrad_src(x: torch.Tensor, mode: int = 0, h0=None, keep=None, T: int = 0):
    if x.stride(-1) != 1:
        x = x.contiguous()
    return x, _native.WgradSrc(x.shape[-1], mode, x.stride(-2), x.data_ptr(), None,
                               h0.data_ptr() if h0 is not None else None,
                               keep.data_ptr() if keep is not None else None, T, 0)


def wgrad(dy: torch.Tensor, sources, with_bias: bool):
    """([dy^T x_k for each source], column sums of dy or None) in one swarm_wgrad launch; sources
    are _wgrad_src() pairs (tensor kept alive, descriptor)."""
    if dy.stride(-1) != 1:
        dy = dy.contiguous()
    rows, out_f = dy.shape
    dws, descs = [], []
    for x, d in sources:
        dw = torch.empty(out_f, d.in_f, dtype=dy.dtype, device=dy.device)
        d.dw = dw.data_ptr()
        dws.append(dw)
        descs.append(d)
    db = torch.empty(out_f, dtype=dy.dtype, device=dy.device) if with_bias else None
    arr = (_native.WgradSrc * len(descs))(*descs)
    lib = _native.load()
    stream = C.c_void_p(torch.cuda.current_stream(dy.device).cuda_stream)
    _native.check(lib.swarm_wgrad(rows, out_f, _ptr(dy), dy.stride(0), len(descs), C.cast(arr, C.c_void_p),
                                  _ptr(db), stream), "swarm_wgrad")
    return dws, db


class _RowsWgradLinear(torch.autograd.Function):
    """y = x W^T [+ x2 W2^T] [+ b] (addmm, as F.linear) whose weight and bias gradients come from
    ONE swarm_wgrad launch (dx, dx2: library GEMMs). x2 / W2 carry a second product into the same
    output, e.g. an LSTM step's [x | h0] [W_ih | W_hh]^T without concatenating either side."""

    @staticmethod
    def forward(ctx, x, weight, bias, x2, weight2):
        y = torch.addmm(bias, x, weight.t()) if bias is not None else x.mm(weight.t())
        if x2 is not None:
            y.addmm_(x2, weight2.t())
        ctx.save_for_backward(x, weight, x2, weight2)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, x2, weight2 = ctx.saved_tensors
        ng = ctx.needs_input_grad
        dy = dy.contiguous()
        dx = dy.mm(weight) if ng[0] else None
        dx2 = dy.mm(weight2) if x2 is not None and ng[3] else None
        srcs = [_wgrad_src(x)] + ([_wgrad_src(x2)] if x2 is not None else [])
        dws, db = wgrad(dy, srcs, ctx.has_bias and ng[2])
        return dx, dws[0] if ng[1] else None, db, dx2, (dws[1] if x2 is not None and ng[4] else None)


def _rows_linear(x2d: torch.Tensor, weight, bias):
    """F.linear over a 2-D input with the weight gradient routed by row count (GPU + autograd)."""
    rows = x2d.shape[0]
    if x2d.is_cuda and torch.is_grad_enabled() and x2d.dtype == torch.float32:
        if rows >= SPLITK_MIN_ROWS:
            return _SplitKLinear.apply(x2d.contiguous(), weight, bias)
        if WGRAD_NATIVE and rows >= WGRAD_MIN_ROWS:
            return _RowsWgradLinear.apply(x2d, weight, bias, None, None)
    return torch.nn.functional.linear(x2d, weight, bias)


class _Linear(nn.Linear):
    """nn.Linear (same parameters and state-dict keys) whose GPU calls with autograd take the
    split-row weight gradient of _SplitKLinear (>= SPLITK_MIN_ROWS rows) or swarm_wgrad
    (>= WGRAD_MIN_ROWS rows)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not (x.is_cuda and torch.is_grad_enabled() and x.dtype == torch.float32):
            return super().forward(x)
        rows = x.numel() // x.shape[-1] if x.dim() else 0
        if rows < WGRAD_MIN_ROWS or (rows < SPLITK_MIN_ROWS and not WGRAD_NATIVE):
            return super().forward(x)
        y = _rows_linear(x.reshape(rows, x.shape[-1]), self.weight, self.bias)
        return y.view(*x.shape[:-1], self.out_features)


class _StackedView(torch.autograd.Function):
    """A stacked parameter storage as a differentiable function of the Parameters that alias it
    (no copy): forward returns the storage itself, backward hands each Parameter its slice of
    the gradient (what the backward of torch.cat over those Parameters would hand them)."""

    @staticmethod
    def forward(ctx, stacked, spans, *params):
        ctx.spans = spans
        return stacked.view_as(stacked)

    @staticmethod
    def backward(ctx, g):
        flat = g.contiguous().reshape(-1)
        return (None, None) + tuple(flat[a:b].view(shape) for a, b, shape in ctx.spans)


class StackedLinears:
    """The weights and biases of several Linear layers with one in_features, moved into one
    (sum out, in) / (sum out,) storage in the given order; each layer's Parameter is re-pointed
    (.data) to its slice, so the Parameter objects (optimizer state, state_dict keys, checkpoints)
    are unchanged while a forward reads the stacked storage instead of concatenating the layers'
    tensors per call (torch.cat: one kernel each for the weights and the biases)."""

    def __init__(self, linears):
        self.linears = list(linears)
        self.restack()

    def restack(self):
        ref = self.linears[0].weight
        H = ref.shape[1]
        outs = [m.out_features for m in self.linears]
        self.W = torch.empty(sum(outs), H, dtype=ref.dtype, device=ref.device)
        self.B = torch.empty(sum(outs), dtype=ref.dtype, device=ref.device)
        w_spans, b_spans, off = [], [], 0
        with torch.no_grad():
            for m, n in zip(self.linears, outs):
                self.W[off:off + n].copy_(m.weight)
                self.B[off:off + n].copy_(m.bias)
                m.weight.data = self.W[off:off + n]
                m.bias.data = self.B[off:off + n]
                w_spans.append((off * H, (off + n) * H, (n, H)))
                b_spans.append((off, off + n, (n,)))
                off += n
        self.w_spans, self.b_spans = tuple(w_spans), tuple(b_spans)

    def intact(self) -> bool:
        """Every Parameter still aliases the storage (a deepcopy or .to() gives them their own)."""
        wp, bp, es = self.W.data_ptr(), self.B.data_ptr(), self.W.element_size()
        return all(m.weight.data_ptr() == wp + a * es and m.bias.data_ptr() == bp + b0 * es
                   for m, (a, _, _), (b0, _, _) in zip(self.linears, self.w_spans, self.b_spans))

    def tensors(self):
        """(W, B) as functions of the layers' Parameters, or None when the aliasing is broken
        inside a graph capture (the caller concatenates); re-stacked here otherwise."""
        if not self.intact():
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                return None
            self.restack()
        return (_StackedView.apply(self.W, self.w_spans, *[m.weight for m in self.linears]),
                _StackedView.apply(self.B, self.b_spans, *[m.bias for m in self.linears]))


def _linear_layer(input_size: int, output_size: int, kernel_init: str = "xavier_uniform",
                  kernel_gain: float = 1.0, bias_init: str = "zeros") -> nn.Linear:
    """ML-Agents-initialised linear layer (poca_networks.py:58-82)."""
    if kernel_init not in _KERNEL_INITS:
        raise ValueError(f"Unknown kernel_init: {kernel_init}")
    layer = _Linear(input_size, output_size)
    _KERNEL_INITS[kernel_init](layer.weight)
    layer.weight.data *= kernel_gain
    if bias_init == "zeros":
        nn.init.zeros_(layer.bias)
    return layer


def _mlagents_lstm(input_size: int, memory_size: int, forget_bias: float = 1.0) -> tuple[nn.LSTM, int]:
    """LSTM with ML-Agents' memory convention (poca_networks.py:85-113): a memory
    vector of `memory_size` holds h and c, i.e. memory_size // 2 units; Xavier per
    gate block, forget-gate bias added to both bias tensors."""
    memory_size = int(memory_size)
    if memory_size <= 0 or memory_size % 2:
        raise ValueError("ML-Agents memory_size must be a positive even integer")
    units = memory_size // 2
    lstm = nn.LSTM(input_size, units, batch_first=True)
    for name, param in lstm.named_parameters():
        gates = param.data.view(4, param.shape[0] // 4, *param.shape[1:])
        if "weight" in name:
            for g in range(4):
                nn.init.xavier_uniform_(gates[g])
        elif "bias" in name:
            nn.init.zeros_(param)
            gates[1].add_(forget_bias)
    return lstm, units


FUSED_LSTM = True   # False: every LSTM call runs torch's nn.LSTM (benchmarks of the reference path)
FUSED_ATTENTION = True   # False: ResidualSelfAttention's core runs torch's bmm / softmax path
# False (or SWARM_FUSED_NORMS=0): its LayerNorms, residual add and set mean run torch's ops
FUSED_NORMS = os.environ.get("SWARM_FUSED_NORMS", "1") != "0"


def _plain_lstm(lstm: nn.LSTM) -> bool:
    return (lstm.num_layers == 1 and not lstm.bidirectional and lstm.batch_first and lstm.proj_size == 0
            and lstm.bias)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class _LSTMSequences(torch.autograd.Function):
    """k independent whole-sequence LSTM recurrences (same length T and unit count) in ONE
    swarm_lstm_seq_forward_batch / _backward_batch launch each way (include/swarmtrain.h).
    Arguments: k, then per problem the gate pre-activations xg = x W_ih^T + b_ih + b_hh
    (n, T, 4U), W_hh, the initial state h0, c0 (n, U) and the optional per-step state mask
    keep (n, T). Returns per problem the hidden sequence (n, T, U) and the final cell
    state (n, U)."""

    @staticmethod
    def forward(ctx, k, *args):
        probs = [args[5 * i:5 * i + 5] for i in range(k)]
        xg0 = probs[0][0]
        T, G = xg0.shape[1], xg0.shape[2]
        U = G // 4
        outs, descs, saved = [], [], []
        for xg, w_hh, h0, c0, keep in probs:
            n = xg.shape[0]
            h_out = torch.empty(n, T, U, dtype=xg.dtype, device=xg.device)
            c_out = torch.empty_like(h_out)
            act = torch.empty_like(xg)
            descs.append(_native.LstmSeqFwd(n, _addr(xg), _addr(w_hh), _addr(h0), _addr(c0), _addr(keep),
                                            _addr(h_out), _addr(c_out), _addr(act)))
            saved += [w_hh, h0, c0, keep, h_out, c_out, act]
        arr = (_native.LstmSeqFwd * k)(*descs)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(xg0.device).cuda_stream)
        _native.check(lib.swarm_lstm_seq_forward_batch(k, T, U, C.cast(arr, C.c_void_p), stream),
                      "swarm_lstm_seq_forward_batch")
        for i in range(k):
            h_out, c_out = saved[7 * i + 4], saved[7 * i + 5]
            outs += [h_out, c_out[:, -1]]     # the final cell state: a view (after the launch that writes c_out)
        ctx.k = k
        ctx.set_materialize_grads(False)   # an unused final state (the update's) gets no zero-filled gradient
        ctx.save_for_backward(*saved)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        k = ctx.k
        saved = ctx.saved_tensors
        # problems none of whose inputs need a gradient (a frozen network's forward run in the
        # same launch) take no part in the backward launch
        live = [i for i in range(k) if any(ctx.needs_input_grad[1 + 5 * i:1 + 5 * i + 4])]
        if not live:
            return (None,) * (1 + 5 * k)
        descs, res, keepalive = [], {}, []
        for i in live:
            w_hh, h0, c0, keep, h_out, c_out, act = saved[7 * i:7 * i + 7]
            dh_out = grads[2 * i].contiguous() if grads[2 * i] is not None else torch.zeros_like(h_out)
            dc_n = grads[2 * i + 1].contiguous() if grads[2 * i + 1] is not None else None
            dxg = torch.empty_like(act)
            dh0, dc0 = torch.empty_like(h0), torch.empty_like(c0)
            descs.append(_native.LstmSeqBwd(h_out.shape[0], _addr(w_hh), _addr(c0), _addr(keep), _addr(c_out),
                                            _addr(act), _addr(dh_out), None, _addr(dc_n), _addr(dxg), _addr(dh0),
                                            _addr(dc0)))
            keepalive += [dh_out, dc_n]
            res[i] = (dxg, dh0, dc0)
        n0, T, U = saved[4].shape
        arr = (_native.LstmSeqBwd * len(live))(*descs)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(saved[4].device).cuda_stream)
        _native.check(lib.swarm_lstm_seq_backward_batch(len(live), T, U, C.cast(arr, C.c_void_p), stream),
                      "swarm_lstm_seq_backward_batch")
        out = [None]
        for i in range(k):
            if i not in res:
                out += [None] * 5
                continue
            w_hh, h0, c0, keep, h_out, c_out, act = saved[7 * i:7 * i + 7]
            dxg, dh0, dc0 = res[i]
            dw = None
            if ctx.needs_input_grad[1 + 5 * i + 1]:
                # W_hh's gradient: dgates^T h_prev' over every (sequence, step) row, one GEMM
                rows = dxg.numel() // (4 * U)
                if WGRAD_NATIVE and rows < SPLITK_MIN_ROWS:
                    # h_prev read in place (h0 at t = 0, else the masked previous step)
                    dw = wgrad(dxg.reshape(rows, 4 * U),
                               [_wgrad_src(h_out.reshape(rows, U), 1, h0, keep, h_out.shape[1])], False)[0][0]
                else:
                    prev = h_out[:, :-1] if keep is None else h_out[:, :-1] * keep[:, :-1, None]
                    h_prev = torch.cat([h0.unsqueeze(1), prev], dim=1)
                    if rows >= SPLITK_MIN_ROWS:   # a 12,288-deep reduction as one GEMM took 134 us
                        dw = _split_rows_weight_grad(dxg.reshape(rows, 4 * U), h_prev.reshape(rows, U), False)[0]
                    else:
                        dw = dxg.reshape(-1, 4 * U).t().mm(h_prev.reshape(-1, U))
            out += [dxg, dw, dh0, dc0, None]
        return tuple(out)


def _addr(t):
    return t.data_ptr() if t is not None else None


class _AttnCore(torch.autograd.Function):
    """softmax((q k^T) / sqrt(D) + key_mask * NEG_INF) v per entity set and head on
    swarm_rsa_attn_forward / _backward (include/swarmtrain.h, v_mfma_f32_16x16x4_f32):
    qkv (S*N, 3D) is the fused q | k | v projection, key_mask (S, N) f32 or None;
    returns att (S*N, D). The backward recomputes the probabilities."""

    @staticmethod
    def forward(ctx, qkv, key_mask, S: int, N: int, H: int):
        D = qkv.shape[1] // 3
        att = torch.empty(S * N, D, dtype=qkv.dtype, device=qkv.device)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
        _native.check(lib.swarm_rsa_attn_forward(S, N, H, D, _ptr(qkv), _ptr(key_mask), _ptr(att), stream),
                      "swarm_rsa_attn_forward")
        ctx.save_for_backward(qkv, key_mask)
        ctx.dims = (S, N, H, D)
        return att

    @staticmethod
    def backward(ctx, d_att):
        qkv, key_mask = ctx.saved_tensors
        S, N, H, D = ctx.dims
        d_qkv = torch.empty_like(qkv)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
        _native.check(lib.swarm_rsa_attn_backward(S, N, H, D, _ptr(qkv), _ptr(key_mask), _ptr(d_att.contiguous()),
                                                  _ptr(d_qkv), stream),
                      "swarm_rsa_attn_backward")
        return d_qkv, None, None, None, None


class _RowNorm(torch.autograd.Function):
    """LayerNorm without affine (eps 1e-5) of (rows, D) on swarm_row_norm_forward / _backward
    (include/swarmtrain.h): the saved x_hat is the output itself, plus 1/std per row."""

    @staticmethod
    def forward(ctx, x):
        rows, D = x.shape
        xhat = torch.empty_like(x)
        rstd = torch.empty(rows, dtype=x.dtype, device=x.device)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _native.check(lib.swarm_row_norm_forward(rows, D, _ptr(x), _ptr(xhat), _ptr(rstd), stream),
                      "swarm_row_norm_forward")
        ctx.save_for_backward(xhat, rstd)
        return xhat

    @staticmethod
    def backward(ctx, dy):
        xhat, rstd = ctx.saved_tensors
        dx = torch.empty_like(xhat)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(xhat.device).cuda_stream)
        _native.check(lib.swarm_row_norm_backward(xhat.shape[0], xhat.shape[1], _ptr(dy.contiguous()), _ptr(xhat),
                                                  _ptr(rstd), _ptr(dx), stream), "swarm_row_norm_backward")
        return dx


class _SetPool(torch.autograd.Function):
    """LayerNorm(a + x).mean over each set of n rows (the residual tail of
    ResidualSelfAttention, poca_networks.py:486-491) in one pass each way on
    swarm_set_pool_forward / _backward: a, x (S*n, D) -> pooled (S, D)."""

    @staticmethod
    def forward(ctx, a, x, S: int, n: int):
        D = a.shape[1]
        xhat = torch.empty_like(a)
        rstd = torch.empty(a.shape[0], dtype=a.dtype, device=a.device)
        pooled = torch.empty(S, D, dtype=a.dtype, device=a.device)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(a.device).cuda_stream)
        _native.check(lib.swarm_set_pool_forward(S, n, D, _ptr(a), _ptr(x), _ptr(xhat), _ptr(rstd), _ptr(pooled),
                                                 stream), "swarm_set_pool_forward")
        ctx.save_for_backward(xhat, rstd)
        ctx.dims = (S, n)
        return pooled

    @staticmethod
    def backward(ctx, dpooled):
        xhat, rstd = ctx.saved_tensors
        S, n = ctx.dims
        dz = torch.empty_like(xhat)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(xhat.device).cuda_stream)
        _native.check(lib.swarm_set_pool_backward(S, n, xhat.shape[1], _ptr(dpooled.contiguous()), _ptr(xhat),
                                                  _ptr(rstd), _ptr(dz), stream), "swarm_set_pool_backward")
        return dz, dz, None, None


def lstm_sequence(lstm: nn.LSTM, seq: torch.Tensor, state, keep: torch.Tensor | None = None):
    """lstm(seq, state) for a batch-first single-layer nn.LSTM, optionally with the
    carried state masked between steps: keep (n, T) multiplies (h, c) after step t
    before step t + 1 — the trainers' per-step loops that zero the memory of rows
    whose episode ended (poca_trainer.py:706-723, option_critic_trainer.py:496-506).
    On the GPU the recurrence is one swarm_lstm_seq_* launch each way (autograd
    supported); elsewhere the reference's loop of nn.LSTM calls."""
    return lstm_sequences([(lstm, seq, state, keep)])[0]


def _fused_seq_ok(lstm: nn.LSTM, seq: torch.Tensor) -> bool:
    return (FUSED_LSTM and seq.is_cuda and _plain_lstm(lstm) and lstm.hidden_size <= _native.LSTM_SEQ_MAX_UNITS
            and seq.dtype == torch.float32)


def lstm_sequences(items):
    """[lstm_sequence(lstm, seq, state, keep) for each item] with the GPU recurrences of items
    that share a sequence length and unit count in ONE launch each way (_LSTMSequences): the
    actor's and the critics' memories of a minibatch are independent, and one launch runs
    their latency-bound chains side by side instead of back to back. An item may carry a fifth
    element `frozen` = True: its forward runs without autograd (as under torch.no_grad, its
    outputs detached) and it takes no part in the backward launch."""
    out = [None] * len(items)
    groups: dict = {}
    for i, item in enumerate(items):
        lstm, seq, state, keep = item[:4]
        if _fused_seq_ok(lstm, seq) and seq.shape[1] == 1 and seq.shape[0] >= SINGLE_STEP_ROWS:
            frozen = len(item) > 4 and item[4]
            with torch.no_grad() if frozen else contextlib.nullcontext():
                out[i] = _lstm_single_step(lstm, seq, state)
        elif _fused_seq_ok(lstm, seq):
            groups.setdefault((seq.shape[1], lstm.hidden_size, seq.device), []).append(i)
        else:
            frozen = len(item) > 4 and item[4]
            with torch.no_grad() if frozen else contextlib.nullcontext():
                out[i] = _lstm_loop(lstm, seq, state, keep)
    for idx in groups.values():
        for chunk in (idx[j:j + _native.LSTM_MAX_BATCH] for j in range(0, len(idx), _native.LSTM_MAX_BATCH)):
            args, frozen_of = [], []
            for i in chunk:
                lstm, seq, state, keep = items[i][:4]
                frozen = len(items[i]) > 4 and items[i][4]
                n, units = seq.shape[0], lstm.hidden_size
                with torch.no_grad() if frozen else contextlib.nullcontext():
                    bias = lstm.bias_ih_l0 + lstm.bias_hh_l0
                    rows = seq.shape[0] * seq.shape[1]
                    if torch.is_grad_enabled() and rows >= WGRAD_MIN_ROWS:
                        xg = _rows_linear(seq.reshape(rows, -1), lstm.weight_ih_l0,
                                          bias).view(seq.shape[0], seq.shape[1], -1)
                    else:
                        xg = torch.nn.functional.linear(seq, lstm.weight_ih_l0, bias)
                    w_hh = lstm.weight_hh_l0.contiguous()
                    h0, c0 = state[0].reshape(n, units).contiguous(), state[1].reshape(n, units).contiguous()
                if frozen:
                    xg, w_hh, h0, c0 = xg.detach(), w_hh.detach(), h0.detach(), c0.detach()
                args += [xg.contiguous(), w_hh, h0, c0, keep.to(torch.float32).contiguous() if keep is not None else None]
                frozen_of.append(frozen)
            res = _LSTMSequences.apply(len(chunk), *args)
            for j, i in enumerate(chunk):
                h_seq, c_n = res[2 * j], res[2 * j + 1]
                if frozen_of[j]:
                    h_seq, c_n = h_seq.detach(), c_n.detach()
                out[i] = (h_seq, (h_seq[:, -1].unsqueeze(0), c_n.unsqueeze(0)))
    return out


# One-step recurrences over at least this many rows (the OC2 update's next-state actor pass:
# 2,048 manager rows and 12,288 option rows per C5 minibatch) leave the whole-sequence kernel,
# whose workgroup per row loads its gate rows of W_hh for a single step (449 us for the 12,288
# option rows), for two library GEMMs and the cell's elementwise terms (autograd-capable).
SINGLE_STEP_ROWS = 512


class _LSTMCell(torch.autograd.Function):
    """c1 = sigmoid(f) c0 + sigmoid(i) tanh(g), h1 = sigmoid(o) tanh(c1) from the gate pre-activations
    (n, 4U) in ONE kernel each way (swarm_lstm_cell / swarm_lstm_cell_backward) instead of torch's
    ~9 elementwise kernels forward and ~15 backward; a missing output gradient stays unmaterialised."""

    @staticmethod
    def forward(ctx, gates, c0):
        gates, c0 = gates.contiguous(), c0.contiguous()
        n, units = c0.shape
        h1, c1 = torch.empty_like(c0), torch.empty_like(c0)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(gates.device).cuda_stream)
        _native.check(lib.swarm_lstm_cell(n, units, _ptr(gates), _ptr(c0), _ptr(h1), _ptr(c1), stream),
                      "swarm_lstm_cell")
        ctx.save_for_backward(gates, c0, c1)
        ctx.set_materialize_grads(False)
        return h1, c1

    @staticmethod
    def backward(ctx, dh, dc):
        gates, c0, c1 = ctx.saved_tensors
        n, units = c0.shape
        dgates, dc0 = torch.empty_like(gates), torch.empty_like(c0)
        dh = dh.contiguous() if dh is not None else None
        dc = dc.contiguous() if dc is not None else None
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(gates.device).cuda_stream)
        _native.check(lib.swarm_lstm_cell_backward(n, units, _ptr(gates), _ptr(c0), _ptr(c1), _ptr(dh), _ptr(dc),
                                                   _ptr(dgates), _ptr(dc0), stream), "swarm_lstm_cell_backward")
        return dgates, dc0


FUSED_LSTM_CELL = os.environ.get("SWARM_LSTM_CELL", "1") != "0"


def _lstm_single_step(lstm: nn.LSTM, seq: torch.Tensor, state):
    """lstm(seq, state) for T = 1 (nn.LSTM's gate order i, f, g, o). A keep mask acts only
    between steps, so a single step has none to apply."""
    n, units = seq.shape[0], lstm.hidden_size
    x, h0 = seq.reshape(n, -1), state[0].reshape(n, units)
    if seq.is_cuda and torch.is_grad_enabled() and n >= SPLITK_MIN_ROWS:
        # [x | h0] [W_ih | W_hh]^T + b as ONE product whose weight gradient takes the split-row
        # reduction (the library's single GEMM for dW_hh over 12,288 rows took 136 us)
        gates = _SplitKLinear.apply(torch.cat([x, h0], dim=1),
                                    torch.cat([lstm.weight_ih_l0, lstm.weight_hh_l0], dim=1),
                                    lstm.bias_ih_l0 + lstm.bias_hh_l0)
    elif seq.is_cuda and torch.is_grad_enabled() and WGRAD_NATIVE and n >= WGRAD_MIN_ROWS:
        # the same two products into one output; dW_ih, dW_hh and the bias gradient in one launch
        gates = _RowsWgradLinear.apply(x, lstm.weight_ih_l0, lstm.bias_ih_l0 + lstm.bias_hh_l0, h0,
                                       lstm.weight_hh_l0)
    else:
        gates = torch.addmm(torch.nn.functional.linear(x, lstm.weight_ih_l0, lstm.bias_ih_l0 + lstm.bias_hh_l0),
                            h0, lstm.weight_hh_l0.t())
    if FUSED_LSTM_CELL and seq.is_cuda and gates.dtype == torch.float32:
        h1, c1 = _LSTMCell.apply(gates, state[1].reshape(n, units))
        return h1.view(n, 1, units), (h1.view(1, n, units), c1.view(1, n, units))
    i, f, g, o = gates.chunk(4, dim=1)
    c1 = torch.sigmoid(f) * state[1].reshape(n, units) + torch.sigmoid(i) * torch.tanh(g)
    h1 = torch.sigmoid(o) * torch.tanh(c1)
    return h1.view(n, 1, units), (h1.view(1, n, units), c1.view(1, n, units))


def _lstm_loop(lstm: nn.LSTM, seq: torch.Tensor, state, keep: torch.Tensor | None = None):
    """The reference's path: nn.LSTM over the sequence, or its per-step masked loop."""
    n, T, _ = seq.shape
    if keep is None:
        return lstm(seq, state)
    outs = []
    for t in range(T):
        o, state = lstm(seq[:, t:t + 1], state)
        outs.append(o)
        if t < T - 1:
            k = keep[:, t].reshape(1, n, 1).to(o.dtype)
            state = (state[0] * k, state[1] * k)
    return torch.cat(outs, dim=1), state


def batched_sequence_passes(requests, extra_items=()):
    """POCACritic.sequence_passes of several critics (requests: (critic, all_states,
    all_actions, focal_agent_ids, memories, sequence_length, passes) each) with all their
    memories, and any `extra_items` (other independent LSTM items), in ONE LSTM launch each
    way. Returns (the values of each request, the outputs of the extra items)."""
    begun = [req[0].sequence_passes_begin(*req[1:]) for req in requests]
    items = [it for it, _ in begun if it is not None] + list(extra_items)
    outs = lstm_sequences(items) if items else []
    values, j = [], 0
    for (critic, *_), (it, ctx) in zip(requests, begun):
        lstm_out = None
        if it is not None:
            lstm_out = outs[j][0]
            j += 1
        values.append(critic.sequence_passes_end(lstm_out, ctx))
    return values, outs[j:]


def _lstm(lstm: nn.LSTM, seq: torch.Tensor, state, keep: torch.Tensor | None = None):
    """lstm(seq, state) for a batch-first single-layer nn.LSTM. Rollout-time calls
    (one step, no autograd, on the GPU) take the fused cell path: the gate
    pre-activations as two library GEMMs, then swarm_lstm_cell
    (include/swarmcritic.h) for the cell update. Every other GPU call (the
    updates' sequences, with autograd) goes through lstm_sequence's
    whole-sequence kernels."""
    n, T, _ = seq.shape
    if not (FUSED_LSTM and T == 1 and keep is None and seq.is_cuda and not torch.is_grad_enabled()
            and _plain_lstm(lstm)):
        return lstm_sequence(lstm, seq, state, keep)
    units = lstm.hidden_size
    h0, c0 = state
    h0 = h0.reshape(n, units)
    c0 = c0.reshape(n, units).contiguous()
    gates = torch.nn.functional.linear(seq.reshape(n, -1), lstm.weight_ih_l0, lstm.bias_ih_l0 + lstm.bias_hh_l0)
    gates.addmm_(h0, lstm.weight_hh_l0.t())
    h1 = torch.empty(1, n, units, dtype=seq.dtype, device=seq.device)
    c1 = torch.empty_like(h1)
    lib = _native.load()
    rc = lib.swarm_lstm_cell(n, units, C.c_void_p(gates.data_ptr()), C.c_void_p(c0.data_ptr()),
                             C.c_void_p(h1.data_ptr()), C.c_void_p(c1.data_ptr()),
                             C.c_void_p(torch.cuda.current_stream(seq.device).cuda_stream))
    _native.check(rc, "swarm_lstm_cell")
    return h1.view(n, 1, units), (h1, c1)


def checkpoint_memory_size(checkpoint: dict, default: int = 128) -> int:
    """Total ML-Agents memory size of a checkpoint (poca_networks.py:116-127):
    checkpoints older than the parity revision stored the LSTM unit count."""
    value = int(checkpoint.get("memory_size", default))
    return value if checkpoint.get("memory_size_semantics") == "mlagents_total" else 2 * value


def _mlp(input_size: int, num_layers: int, hidden: int, kernel_init: str, kernel_gain: float = 1.0):
    dims = [input_size] + [hidden] * num_layers
    mods: list[nn.Module] = []
    for a, b in zip(dims[:-1], dims[1:]):
        mods += [_linear_layer(a, b, kernel_init=kernel_init, kernel_gain=kernel_gain), Swish()]
    return nn.Sequential(*mods)


class LinearEncoder(nn.Module):
    """Linear + Swish stack (poca_networks.py:133-170)."""

    def __init__(self, input_size: int, num_layers: int, hidden_size: int, kernel_init: str = "kaiming_normal",
                 kernel_gain: float = 1.0):
        super().__init__()
        self.net = _mlp(input_size, num_layers, hidden_size, kernel_init, kernel_gain)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)


class EntityEmbedding(nn.Module):
    """One-layer entity encoder with T-Fixup init (poca_networks.py:173-194)."""

    def __init__(self, entity_size: int, embedding_size: int):
        super().__init__()
        self.encoder = LinearEncoder(entity_size, 1, embedding_size, kernel_init="normal",
                                     kernel_gain=(0.125 / embedding_size) ** 0.5)

    def forward(self, entities: torch.Tensor) -> torch.Tensor:
        return self.encoder(entities)


class Actor(nn.Module):
    """Gaussian actor, state-independent log-std, per-dimension log-probs
    (poca_networks.py:197-257)."""

    def __init__(self, obs_dim: int, act_dim: int, hidden: int = 256, num_layers: int = 2):
        super().__init__()
        self.net = _mlp(obs_dim, num_layers, hidden, "kaiming_normal")
        self.mu_head = _linear_layer(hidden, act_dim, kernel_init="kaiming_normal", kernel_gain=0.2)
        self.log_std = nn.Parameter(torch.zeros(1, act_dim))

    def forward(self, obs: torch.Tensor):
        mu = self.mu_head(self.net(obs))
        return mu, (mu * 0 + self.log_std).exp()

    def get_dist(self, obs: torch.Tensor) -> Normal:
        return Normal(*self(obs), validate_args=False)

    def evaluate(self, obs: torch.Tensor, actions: torch.Tensor):
        dist = self.get_dist(obs)
        return dist.log_prob(actions), dist.entropy().mean(dim=-1)


class DiscreteActor(nn.Module):
    """Categorical actor over behaviour modules (poca_networks.py:260-314)."""

    def __init__(self, obs_dim: int, num_actions: int, hidden: int = 256, num_layers: int = 2):
        super().__init__()
        self.num_actions = num_actions
        self.net = _mlp(obs_dim, num_layers, hidden, "kaiming_normal")
        self.logits_head = _linear_layer(hidden, num_actions, kernel_init="kaiming_normal", kernel_gain=0.1)

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        return self.logits_head(self.net(obs))

    def get_dist(self, obs: torch.Tensor) -> torch.distributions.Categorical:
        return torch.distributions.Categorical(validate_args=False, logits=self(obs))

    def evaluate(self, obs: torch.Tensor, actions: torch.Tensor):
        dist = self.get_dist(obs)
        return dist.log_prob(actions.squeeze(-1).long()).unsqueeze(-1), dist.entropy()


class RecurrentDiscreteActor(nn.Module):
    """Categorical actor with an LSTM memory, the cyclamen policy (poca_networks.py:320-414)."""

    def __init__(self, obs_dim: int, num_actions: int, hidden: int = 128, num_layers: int = 1,
                 memory_size: int = 128):
        super().__init__()
        self.obs_dim, self.num_actions, self.memory_size = obs_dim, num_actions, memory_size
        self.net = LinearEncoder(obs_dim, num_layers, hidden, kernel_init="kaiming_normal")
        self.lstm, self.hidden_size = _mlagents_lstm(hidden, memory_size)
        self.logits_head = _linear_layer(self.hidden_size, num_actions, kernel_init="kaiming_normal",
                                         kernel_gain=0.1)

    def initial_state(self, batch_size: int, device):
        z = torch.zeros(1, batch_size, self.hidden_size, device=device)
        return z, z.clone()

    def forward_sequence(self, obs_seq: torch.Tensor, state=None, keep: torch.Tensor | None = None):
        """(B, T, obs) -> logits (B, T, A), memory. keep (B, T): the memory is multiplied by
        keep[:, t] after step t (the trainer's per-step episode-end resets)."""
        out, nxt = _lstm(*self.sequence_lstm_item(obs_seq, state, keep))
        return self.logits_head(out), nxt

    def sequence_lstm_item(self, obs_seq: torch.Tensor, state=None, keep: torch.Tensor | None = None):
        """forward_sequence up to its LSTM: (lstm, encoded sequence, state, keep), for
        lstm_sequences to run together with other independent memories; the logits are
        logits_head(the LSTM output)."""
        B, T = obs_seq.shape[:2]
        enc = self.net(obs_seq.reshape(B * T, self.obs_dim)).view(B, T, -1)
        return self.lstm, enc, state if state is not None else self.initial_state(B, obs_seq.device), keep

    def step(self, obs: torch.Tensor, state=None):
        logits, nxt = self.forward_sequence(obs.unsqueeze(1), state)
        return logits[:, 0], nxt

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        return self.step(obs)[0]

    def get_dist(self, obs: torch.Tensor, state=None) -> torch.distributions.Categorical:
        return torch.distributions.Categorical(validate_args=False, logits=self.step(obs, state)[0])

    def evaluate_sequence(self, obs_seq: torch.Tensor, actions_seq: torch.Tensor, state=None):
        B, T = obs_seq.shape[:2]
        logits, _ = self.forward_sequence(obs_seq, state)
        dist = torch.distributions.Categorical(validate_args=False, logits=logits.reshape(B * T, self.num_actions))
        act = actions_seq.reshape(B * T, -1).squeeze(-1).long()
        return dist.log_prob(act).view(B, T, 1), dist.entropy().view(B, T)

    def evaluate(self, obs: torch.Tensor, actions: torch.Tensor):
        lp, ent = self.evaluate_sequence(obs.unsqueeze(1), actions.unsqueeze(1))
        return lp[:, 0], ent[:, 0]


class ResidualSelfAttention(nn.Module):
    """Pre-norm multi-head self-attention + residual + masked mean pooling
    (poca_networks.py:417-491); LayerNorms without affine parameters, logits
    scaled by sqrt(embed_dim)."""

    NEG_INF = -1e6
    EPSILON = 1e-7

    def __init__(self, embed_dim: int, num_heads: int = 4):
        super().__init__()
        assert embed_dim % num_heads == 0
        self.num_heads, self.head_dim, self.embed_dim = num_heads, embed_dim // num_heads, embed_dim
        gain = (0.125 / embed_dim) ** 0.5
        for name in ("fc_q", "fc_k", "fc_v", "fc_out"):
            setattr(self, name, _linear_layer(embed_dim, embed_dim, kernel_init="normal", kernel_gain=gain))
        self.embedding_norm = nn.LayerNorm(embed_dim, elementwise_affine=False)
        self.residual_norm = nn.LayerNorm(embed_dim, elementwise_affine=False)
        # q | k | v in one storage (one projection GEMM without concatenating the weights)
        self.__dict__["_qkv"] = StackedLinears([self.fc_q, self.fc_k, self.fc_v])

    def qkv_params(self, grad: bool = True):
        """(W_q | W_k | W_v, b_q | b_k | b_v): the stacked storage (with autograd through the layers'
        Parameters when `grad`), or their concatenation when the storage cannot be used."""
        if not grad:
            if self._qkv.intact():
                return self._qkv.W, self._qkv.B
        else:
            wb = self._qkv.tensors()
            if wb is not None:
                return wb
        return (torch.cat([self.fc_q.weight, self.fc_k.weight, self.fc_v.weight]),
                torch.cat([self.fc_q.bias, self.fc_k.bias, self.fc_v.bias]))

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        if "_qkv" in self.__dict__:
            self._qkv.restack()
        return out

    def _native_core(self, inp: torch.Tensor) -> bool:
        B, N, D = inp.shape
        return (FUSED_ATTENTION and inp.is_cuda and inp.dtype == torch.float32 and B > 0
                and 1 <= N <= _native.ATTN_MAX_ENTITIES and self.head_dim in _native.ATTN_HEAD_DIMS)

    def forward(self, inp: torch.Tensor, key_mask: torch.Tensor | None = None) -> torch.Tensor:
        B, N, D = inp.shape
        H, d = self.num_heads, self.head_dim
        if self._native_core(inp) and FUSED_NORMS and key_mask is None and D in _native.NORM_WIDTHS:
            # both LayerNorms, the residual add and the set mean on swarm_row_norm_* /
            # swarm_set_pool_* (one pass each way instead of torch's layer_norm / add / mean)
            x2 = _RowNorm.apply(inp.reshape(B * N, D).contiguous())
            w, b = self.qkv_params(torch.is_grad_enabled())
            if torch.is_grad_enabled() and B * N >= SPLITK_MIN_ROWS:
                qkv = _SplitKLinear.apply(x2, w, b)
            else:
                qkv = torch.nn.functional.linear(x2, w, b).contiguous()
            att = _AttnCore.apply(qkv, None, B, N, H)
            return _SetPool.apply(self.fc_out(att).contiguous(), x2, B, N)
        x = self.embedding_norm(inp)
        if self._native_core(inp):
            # the three projections as one GEMM (q | k | v column blocks), then the attention
            # core of every set and head in one MFMA kernel each way (_AttnCore)
            w, b = self.qkv_params(torch.is_grad_enabled())
            x2 = x.reshape(B * N, D)
            if torch.is_grad_enabled() and B * N >= SPLITK_MIN_ROWS:
                qkv = _SplitKLinear.apply(x2, w, b)
            else:
                qkv = torch.nn.functional.linear(x2, w, b).contiguous()
            km = key_mask.reshape(B, N).to(torch.float32).contiguous() if key_mask is not None else None
            att = _AttnCore.apply(qkv, km, B, N, H).view(B, N, D)
        else:
            heads = [f(x).view(B, N, H, d).transpose(1, 2) for f in (self.fc_q, self.fc_k, self.fc_v)]
            logits = (heads[0] @ heads[1].transpose(-2, -1)) / math.sqrt(D)
            if key_mask is not None:
                logits = logits + key_mask.view(B, 1, 1, N) * self.NEG_INF
            att = (logits.softmax(dim=-1) @ heads[2]).transpose(1, 2).contiguous().view(B, N, D)
        out = self.residual_norm(self.fc_out(att) + x)
        if key_mask is None:
            return out.mean(dim=1)
        keep = (1.0 - key_mask).unsqueeze(-1)
        return (out * keep).sum(dim=1) / (keep.sum(dim=1) + self.EPSILON)


def _fused_rsa(attn: ResidualSelfAttention, rows: torch.Tensor, mode, n: int):
    """Attention pooling of the entity sets of every env through swarm_rsa_pool.
    rows: (B, R, h) embedded entities (R = n, or 2n for the baseline sets). `mode`
    may be a tuple of modes over the same rows: the LayerNorm and projection run
    once and a tuple of pooled tensors is returned."""
    modes = mode if isinstance(mode, tuple) else (mode,)
    B = rows.shape[0]
    rows = rows.contiguous()
    x = torch.empty_like(rows)
    lib = _native.load()
    stream = C.c_void_p(torch.cuda.current_stream(rows.device).cuda_stream)
    _native.check(lib.swarm_rsa_embedding_norm(rows.numel() // attn.embed_dim, attn.embed_dim,
                                               C.c_void_p(rows.data_ptr()), C.c_void_p(x.data_ptr()), stream),
                  "swarm_rsa_embedding_norm")
    w, b = attn.qkv_params(torch.is_grad_enabled())
    qkv = torch.nn.functional.linear(x, w, b).contiguous()
    wo, bo = attn.fc_out.weight.contiguous(), attn.fc_out.bias.contiguous()
    out = []
    for m in modes:
        n_sets = n if m == _native.RSA_BASELINES else 1
        pooled = torch.empty(B * n_sets, attn.embed_dim, dtype=torch.float32, device=rows.device)
        rc = lib.swarm_rsa_pool(m, B, n, attn.num_heads, attn.embed_dim, C.c_void_p(x.data_ptr()),
                                C.c_void_p(qkv.data_ptr()), C.c_void_p(wo.data_ptr()), C.c_void_p(bo.data_ptr()),
                                C.c_void_p(pooled.data_ptr()), stream)
        _native.check(rc, "swarm_rsa_pool")
        out.append(pooled)
    return tuple(out) if isinstance(mode, tuple) else out[0]


class POCACritic(nn.Module):
    """Centralised attention critic over the 5-D polar agent states with
    counterfactual baselines (poca_networks.py:506-882)."""

    FUSED_HIDDEN = 128
    FUSED_HEADS = (1, 2, 4)
    FUSED_MAX_ENTITIES = 20

    def __init__(self, state_dim: int, act_dim: int, num_agents: int, h_size: int = 256, num_heads: int = 4,
                 num_layers: int = 2, memory_size: int = 0):
        super().__init__()
        self.state_dim, self.act_dim, self.num_agents, self.h_size = state_dim, act_dim, num_agents, h_size
        self.memory_size = int(memory_size or 0)
        self.obs_entity_enc = EntityEmbedding(state_dim, h_size)
        self.obs_act_entity_enc = EntityEmbedding(state_dim + act_dim, h_size)
        self.self_attn = ResidualSelfAttention(h_size, num_heads)
        self.linear_encoder = LinearEncoder(h_size, num_layers, h_size, kernel_init="kaiming_normal",
                                            kernel_gain=(0.125 / h_size) ** 0.5)
        if self.memory_size > 0:
            self.lstm, self.hidden_size = _mlagents_lstm(h_size, self.memory_size)
        else:
            self.lstm, self.hidden_size = None, h_size
        self.value_head = _linear_layer(self.hidden_size + 1, 1, kernel_init="xavier_uniform")
        self._current_max_agents = nn.Parameter(torch.tensor(1.0), requires_grad=False)
        self.use_fused = True  # set False to force the PyTorch path (benchmarks, debugging)

    # ------------------------------------------------------------ helpers
    def _norm_agent_count(self, n: int, B: int, device) -> torch.Tensor:
        """n in [-1, 1] against the largest n seen (poca_networks.py:579-584). The running
        max is mirrored on the host, keyed by the parameter's version counter (any in-place
        write, incl. load_state_dict, re-reads it), so a pass does not synchronise with the
        device (and can be captured in a graph)."""
        t = self._current_max_agents
        cached = getattr(self, "_max_agents_host", None)
        if cached is None or cached[0] != t._version:
            cached = (t._version, float(t.item()))
        m = cached[1]
        if n > m:
            t.data.fill_(float(n))
            m = float(n)
            cached = (t._version, m)
        self._max_agents_host = cached
        return torch.full((B, 1), n * 2.0 / m - 1.0, device=device)

    def initial_state(self, batch_size: int, device):
        if self.lstm is None:
            return None
        z = torch.zeros(1, batch_size, self.hidden_size, device=device)
        return z, z.clone()

    def _fused(self, ref: torch.Tensor, n_entities: int) -> bool:
        return (self.use_fused and ref.is_cuda and not torch.is_grad_enabled()
                and self.h_size == self.FUSED_HIDDEN and self.self_attn.num_heads in self.FUSED_HEADS
                and 1 <= n_entities <= self.FUSED_MAX_ENTITIES)

    def _value_tail(self, pooled, n_agents, memory=None, sequence_length=1, return_memory=False):
        """linear encoder -> [LSTM] -> agent count -> value head (poca_networks.py:608-625)."""
        B = pooled.shape[0]
        encoding, item = self._tail_begin(pooled, memory, sequence_length)
        next_memory = memory
        if item is not None:
            seq, next_memory = _lstm(*item)
            encoding = seq.reshape(B, self.hidden_size)
        value = self._tail_end(encoding, n_agents)
        return (value, next_memory) if return_memory else value

    def _tail_begin(self, pooled, memory=None, sequence_length=1):
        """The value tail up to its LSTM: (encoding, LSTM item (lstm, sequences, state, None)
        or None without a memory)."""
        B = pooled.shape[0]
        encoding = self.linear_encoder(pooled)
        if self.lstm is None:
            return encoding, None
        sequence_length = int(sequence_length)
        if sequence_length <= 0 or B % sequence_length:
            raise ValueError("Critic batch must be divisible by sequence_length")
        n_seq = B // sequence_length
        return encoding, (self.lstm, encoding.view(n_seq, sequence_length, self.h_size),
                          memory if memory is not None else self.initial_state(n_seq, encoding.device), None)

    def _tail_end(self, encoding, n_agents):
        B = encoding.shape[0]
        encoding = torch.cat([encoding, self._norm_agent_count(n_agents, B, encoding.device)], dim=-1)
        return self.value_head(encoding)

    def _encode_and_value(self, entities, n_agents, memory=None, sequence_length=1, return_memory=False):
        """RSA -> tail on explicit entity sets (B, n, h) (poca_networks.py:597-625)."""
        if self._fused(entities, entities.shape[1]):
            pooled = _fused_rsa(self.self_attn, entities, _native.RSA_SINGLE, entities.shape[1])
        else:
            pooled = self.self_attn(entities)
        return self._value_tail(pooled, n_agents, memory, sequence_length, return_memory)

    # ------------------------------------------------------------ public API
    def critic_pass(self, all_agent_states, memory=None, sequence_length: int = 1, return_memory: bool = False):
        """V(s) from the state-only entities of all agents (poca_networks.py:629-645)."""
        N = all_agent_states.shape[1]
        return self._encode_and_value(self.obs_entity_enc(all_agent_states), N, memory, sequence_length,
                                      return_memory)

    def joint_action_pass(self, all_agent_states, all_agent_actions, memory=None, sequence_length: int = 1,
                          return_memory: bool = False):
        """Q(s, a) over state+action entities (poca_networks.py:647-668)."""
        N = all_agent_states.shape[1]
        ents = self.obs_act_entity_enc(torch.cat([all_agent_states, all_agent_actions], dim=-1))
        return self._encode_and_value(ents, N, memory, sequence_length, return_memory)

    def all_discrete_counterfactual_values(self, all_agent_states, action_indices, num_actions: int):
        """Q for every discrete alternative of every agent, peers fixed (poca_networks.py:670-713)."""
        B, N, _ = all_agent_states.shape
        alts = torch.arange(num_actions, device=all_agent_states.device)
        states = all_agent_states.unsqueeze(1).expand(B, num_actions, N, self.state_dim).reshape(
            B * num_actions, N, self.state_dim)
        out = []
        for agent in range(N):
            idx = action_indices.unsqueeze(1).expand(B, num_actions, N).clone()
            idx[:, :, agent] = alts.unsqueeze(0)
            onehot = torch.nn.functional.one_hot(idx.reshape(B * num_actions, N).long(),
                                                 num_classes=num_actions).to(all_agent_states.dtype)
            out.append(self.joint_action_pass(states, onehot).reshape(B, num_actions))
        return torch.stack(out, dim=1)

    def focal_discrete_counterfactual_values(self, all_agent_states, action_indices, focal_agent_ids,
                                             num_actions: int, memory=None):
        """Q for every alternative of one focal agent per row (poca_networks.py:715-762)."""
        B, N, _ = all_agent_states.shape
        dev = all_agent_states.device
        if self._fused(all_agent_states, N) and N + num_actions <= _native.RSA_MAX_ROWS and B > 0:
            return self._focal_values_shared(all_agent_states, action_indices, focal_agent_ids, num_actions, memory)
        idx = action_indices.unsqueeze(1).expand(B, num_actions, N).clone()
        idx[torch.arange(B, device=dev).unsqueeze(1), torch.arange(num_actions, device=dev).unsqueeze(0),
            focal_agent_ids.long().unsqueeze(1).expand(-1, num_actions)] = \
            torch.arange(num_actions, device=dev).unsqueeze(0)
        onehot = torch.nn.functional.one_hot(idx.reshape(B * num_actions, N).long(),
                                             num_classes=num_actions).to(all_agent_states.dtype)
        states = all_agent_states.unsqueeze(1).expand(B, num_actions, N, self.state_dim).reshape(
            B * num_actions, N, self.state_dim)
        mem = None
        if memory is not None:
            mem = tuple(m.unsqueeze(2).expand(-1, -1, num_actions, -1).reshape(m.shape[0], B * num_actions,
                                                                               m.shape[-1]) for m in memory)
        return self.joint_action_pass(states, onehot, memory=mem).reshape(B, num_actions)

    def _focal_values_shared(self, all_agent_states, action_indices, focal_agent_ids, num_actions: int, memory):
        """focal_discrete_counterfactual_values without re-embedding the A copies of each row's
        set: the N joint entities and the focal robot's A alternative entities are embedded once
        (A + N rows per row, instead of A * N) and swarm_rsa_pool_focal attends the A sets over
        them, sharing the projections and the logits of the row (no-grad, the termination
        advantage's pass). Same sets, same member order as the reference's; only the summation
        order of the shared products differs (float32 rounding)."""
        B, N, S = all_agent_states.shape
        A = num_actions
        dev = all_agent_states.device
        focal = focal_agent_ids.long().reshape(B)
        onehot = torch.nn.functional.one_hot(action_indices.long(), num_classes=A).to(all_agent_states.dtype)
        focal_state = all_agent_states[torch.arange(B, device=dev), focal]
        alt = torch.cat([focal_state.unsqueeze(1).expand(B, A, S),
                         torch.eye(A, dtype=all_agent_states.dtype, device=dev).unsqueeze(0).expand(B, A, A)], dim=-1)
        rows = self.obs_act_entity_enc(torch.cat([torch.cat([all_agent_states, onehot], dim=-1), alt], dim=1))
        rows = rows.contiguous()
        attn = self.self_attn
        x = torch.empty_like(rows)
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _native.check(lib.swarm_rsa_embedding_norm(rows.numel() // attn.embed_dim, attn.embed_dim,
                                                   C.c_void_p(rows.data_ptr()), C.c_void_p(x.data_ptr()), stream),
                      "swarm_rsa_embedding_norm")
        w, b = attn.qkv_params(torch.is_grad_enabled())
        qkv = torch.nn.functional.linear(x, w, b).contiguous()
        wo, bo = attn.fc_out.weight.contiguous(), attn.fc_out.bias.contiguous()
        focal = focal.contiguous()
        pooled = torch.empty(B * A, attn.embed_dim, dtype=torch.float32, device=dev)
        _native.check(lib.swarm_rsa_pool_focal(B, N, A, attn.num_heads, attn.embed_dim, C.c_void_p(x.data_ptr()),
                                               C.c_void_p(qkv.data_ptr()), C.c_void_p(wo.data_ptr()),
                                               C.c_void_p(bo.data_ptr()), C.c_void_p(focal.data_ptr()),
                                               C.c_void_p(pooled.data_ptr()), stream), "swarm_rsa_pool_focal")
        mem = None
        if memory is not None:
            mem = tuple(m.unsqueeze(2).expand(-1, -1, A, -1).reshape(m.shape[0], B * A, m.shape[-1]) for m in memory)
        return self._value_tail(pooled, N, mem).reshape(B, A)

    def baseline(self, agent_i_state, other_states, other_actions, memory=None, sequence_length: int = 1,
                 return_memory: bool = False):
        """Counterfactual b_i: agent i state-only, the others state+action (poca_networks.py:764-788)."""
        M = other_states.shape[1]
        ents = torch.cat([self.obs_entity_enc(agent_i_state.unsqueeze(1)),
                          self.obs_act_entity_enc(torch.cat([other_states, other_actions], dim=-1))], dim=1)
        return self._encode_and_value(ents, 1 + M, memory, sequence_length, return_memory)

    def focal_baselines(self, all_states, all_actions, focal_agent_ids, memory=None, sequence_length: int = 1,
                        return_memory: bool = False):
        """One baseline per row for its focal agent (poca_networks.py:790-820)."""
        B, N, _ = all_states.shape
        rows = torch.arange(B, device=all_states.device)
        focal = focal_agent_ids.long()
        # the other agents in increasing order, as the reference's boolean-mask select, by
        # index (no device -> host sync): other k = k + (k >= focal)
        k = torch.arange(N - 1, device=all_states.device).unsqueeze(0)
        others = (k + (k >= focal.unsqueeze(1)).long()).unsqueeze(-1)
        return self.baseline(all_states[rows, focal],
                             all_states.gather(1, others.expand(B, N - 1, all_states.shape[-1])),
                             all_actions.gather(1, others.expand(B, N - 1, all_actions.shape[-1])), memory,
                             sequence_length, return_memory)

    def _focal_entities(self, all_states, all_actions, focal_agent_ids):
        """The baseline set of each row's focal agent (poca_networks.py:764-820): its state-only
        entity, then the other agents' state+action entities in increasing order (by index,
        no boolean-mask select: other k = k + (k >= focal))."""
        B, N, _ = all_states.shape
        rows = torch.arange(B, device=all_states.device)
        focal = focal_agent_ids.long()
        k = torch.arange(N - 1, device=all_states.device).unsqueeze(0)
        others = (k + (k >= focal.unsqueeze(1)).long()).unsqueeze(-1)
        o_states = all_states.gather(1, others.expand(B, N - 1, all_states.shape[-1]))
        o_actions = all_actions.gather(1, others.expand(B, N - 1, all_actions.shape[-1]))
        return torch.cat([self.obs_entity_enc(all_states[rows, focal].unsqueeze(1)),
                          self.obs_act_entity_enc(torch.cat([o_states, o_actions], dim=-1))], dim=1)

    def sequence_passes(self, all_states, all_actions, focal_agent_ids, memories: dict, sequence_length: int,
                        passes=("value", "baseline")):
        """Several of the critic's training-time passes over the same rows as ONE batched pass:
        "value" = critic_pass(states), "joint" = joint_action_pass(states, actions), "baseline" =
        focal_baselines(states, actions, focal) (poca_trainer.py:748-770, option_critic_trainer.py:
        571-608), each with its own memory (memories[name] = (h, c) of shape (1, sequences, units)).
        Every op of a pass is per set row (self-attention within a set, row-wise encoder and head)
        or per sequence (the LSTM), so stacking the passes along the batch gives each pass's values
        unchanged (up to GEMM summation order): one attention, one encoder, ONE LSTM launch over
        all passes' sequences and one head instead of one of each per pass. Returns the (B,)
        values of each pass in `passes` order."""
        item, ctx = self.sequence_passes_begin(all_states, all_actions, focal_agent_ids, memories, sequence_length,
                                               passes)
        return self.sequence_passes_end(_lstm(*item)[0] if item is not None else None, ctx)

    def sequence_passes_begin(self, all_states, all_actions, focal_agent_ids, memories: dict, sequence_length: int,
                              passes=("value", "baseline")):
        """sequence_passes up to its LSTM: (LSTM item (lstm, sequences, state, None) or None,
        context for sequence_passes_end). With lstm_sequences the item runs in the same launch
        as other independent memories (the actor's)."""
        B, N, _ = all_states.shape
        for name in passes:
            if name not in ("value", "joint", "baseline"):
                raise ValueError(f"unknown critic pass {name!r}")
        sets = []
        for name in passes:
            if name == "value":
                sets.append(self.obs_entity_enc(all_states))
            elif name == "joint":
                sets.append(self.obs_act_entity_enc(torch.cat([all_states, all_actions], dim=-1)))
            else:
                sets.append(self._focal_entities(all_states, all_actions, focal_agent_ids))
        # one pass: its tensors as they are (torch.cat of a single tensor is a copy launch)
        ents = torch.cat(sets, dim=0) if len(sets) > 1 else sets[0]
        memory = None
        if self.lstm is not None:
            memory = tuple(torch.cat([memories[name][i] for name in passes], dim=1) if len(passes) > 1
                           else memories[passes[0]][i] for i in (0, 1))
        pooled = self.self_attn(ents)
        encoding, item = self._tail_begin(pooled, memory, sequence_length)
        return item, (encoding, N, B)

    def sequence_passes_end(self, lstm_out, ctx):
        """The values of sequence_passes from the LSTM output of its item (None without memory)."""
        encoding, N, B = ctx
        if lstm_out is not None:
            encoding = lstm_out.reshape(encoding.shape[0], self.hidden_size)
        return list(self._tail_end(encoding, N).squeeze(-1).split(B))

    def decision_passes(self, all_states, all_actions, *, value: bool = True, joint: bool = False,
                        baselines: bool = True, value_memory=None, joint_memory=None, baseline_memory=None):
        """The per-decision critic calls of the trainers' rollouts on ONE decision's entities:
        V(s) = critic_pass(states, value_memory, return_memory=True), Q(s, a) =
        joint_action_pass(states, actions, joint_memory, return_memory=True) and the baselines
        all_baselines(states, actions, baseline_memory, return_memory=True)
        (poca_trainer.py:519-548, option_critic_trainer.py:330-352,
        learned_option_critic_trainer.py:766-789). Returns a 3-tuple with None for the passes
        not asked for. On the fused path the 2N entity rows of an env are embedded,
        normalised and projected ONCE and every pass is one swarm_rsa_pool launch over them
        (SINGLE_OF_PAIRS, ACTIONS_OF_PAIRS, BASELINES)."""
        B, N, _ = all_states.shape
        if not (joint or baselines):
            return (self.critic_pass(all_states, value_memory, return_memory=True) if value else None), None, None
        if not self._fused(all_states, N):
            return (self.critic_pass(all_states, value_memory, return_memory=True) if value else None,
                    self.joint_action_pass(all_states, all_actions, joint_memory, return_memory=True)
                    if joint else None,
                    self.all_baselines(all_states, all_actions, baseline_memory, return_memory=True)
                    if baselines else None)
        obs_emb = self.obs_entity_enc(all_states)
        act_emb = self.obs_act_entity_enc(torch.cat([all_states, all_actions], dim=-1))
        modes = [m for m, on in ((_native.RSA_SINGLE_OF_PAIRS, value), (_native.RSA_ACTIONS_OF_PAIRS, joint),
                                 (_native.RSA_BASELINES, baselines)) if on]
        pooled = list(_fused_rsa(self.self_attn, torch.cat([obs_emb, act_emb], dim=1), tuple(modes), N))
        out = []
        for on, mem in ((value, value_memory), (joint, joint_memory)):
            out.append(self._value_tail(pooled.pop(0), N, mem, 1, True) if on else None)
        if baselines:
            bl, next_bm = self._value_tail(pooled.pop(0), N, baseline_memory, 1, True)
            out.append((bl.squeeze(-1).reshape(B, N), next_bm))
        else:
            out.append(None)
        return tuple(out)

    def value_and_baselines(self, all_states, all_actions, memory=None, baseline_memory=None):
        """(critic_pass(states, memory, return_memory=True), all_baselines(states, actions,
        baseline_memory, return_memory=True)) — the two critic calls of a POCA rollout
        decision (poca_trainer.py:519-548), through decision_passes."""
        v, _, b = self.decision_passes(all_states, all_actions, value_memory=memory, baseline_memory=baseline_memory)
        return v, b

    def all_baselines(self, all_states, all_actions, memory=None, sequence_length: int = 1,
                      return_memory: bool = False):
        """Baselines of every agent in one pass (poca_networks.py:822-882): set (b, i)
        = [state-only entity i, state+action entities j != i in increasing j]."""
        B, N, _ = all_states.shape
        obs_emb = self.obs_entity_enc(all_states)
        act_emb = self.obs_act_entity_enc(torch.cat([all_states, all_actions], dim=-1))
        if self._fused(all_states, N):
            pooled = _fused_rsa(self.self_attn, torch.cat([obs_emb, act_emb], dim=1), _native.RSA_BASELINES, N)
        else:
            # peers of set i: entities j != i in increasing j (the reference's ~eye mask), by
            # index: j = k + (k >= i), so no boolean-mask select (device -> host sync)
            i = torch.arange(N, device=all_states.device).unsqueeze(1)
            k = torch.arange(N - 1, device=all_states.device).unsqueeze(0)
            peers = act_emb[:, k + (k >= i).long()]                      # (B, N, N - 1, h)
            sets = torch.cat([obs_emb.unsqueeze(2), peers], dim=2).reshape(B * N, N, self.h_size)
            pooled = self.self_attn(sets)
        result = self._value_tail(pooled, N, memory, sequence_length, return_memory)
        if return_memory:
            values, next_memory = result
            return values.squeeze(-1).reshape(B, N), next_memory
        return result.squeeze(-1).reshape(B, N)
