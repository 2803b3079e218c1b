"""BoostedNeuralLDPCDecoder (Kwak et al. 2023) on MI355X.

Reference: src/boosted_neural_ldpc_decoder/BoostedNeuralLDPCDecoder.py:14-538.  Same constructor,
parameter registry (`weight_{CN|UCN|VN}_{iteration}`, shapes by sharing code), helper methods
(fetch_param, get_trainable_parameters, _apply_constraints, _quantize_message) and forward contract
(target_iter / fixed_iter / fixed_iter_weight, module-owned `self.outputs` list).  The decoding loop
(VN weighting + quantisation, UCN flags, min-sum / quantised min-sum / sum-product check nodes,
weight sharing, clipping, marginalisation) runs as HIP kernels (nldpc.decode); the learned weights
get their gradients from nldpc_backward.

What is different from the reference and why:
  * no dense routing buffers are registered (W_*, Lift_Matrix*: 22.9 GB each at z=384); their keys
    in an old state_dict are ignored on load;
  * `self.llr[t]` holds the message state in the kernel layout [B, E, Z] (reference [B, Z, E]); None
    is the initial all-zero state.  The fused kernel keeps the state on chip, so inside a run of
    consecutive iterations the boundaries are recorded (input, weights, starting state) and the state
    is recomputed on demand -- the value the reference stored -- when a later call resumes there
    (e.g. forward() followed by forward(target_iter=k)).  The record holds its own copy of the
    channel input and of the previous posterior (UCN), so a caller that refills its xa buffer in place
    between the calls still resumes from the state the reference stored (Boosted…py:512); a starting
    state modified in place is detected (tensor version) and raises.  Such a recomputed state is a
    constant: a gradient does not flow back into the call that produced it (in the reference it would
    reach that call's graph, which a completed backward has already freed).  The final boundary of a
    call, self.llr[last + 1], is that call's own output state and stays attached to its graph, as the
    reference's self.llr[t + 1] does: resuming from it after a completed backward fails the same way
    in both ("backward through the graph a second time").  Exception: when that boundary is
    self.llr[T] (the call ran up to the last iteration), no later call can resume from it, so the
    fused kernel does not write it (65 536 codewords x E x Z = 19.8 GB at BG2 z=384) and it is
    recomputed on demand, as a constant, if read.
  * gradients flow through the message state between the segments of one call (list-valued xa: one
    segment per iteration; split iteration lists), as through the reference's self.llr[t + 1].
"""
import dataclasses
from typing import Optional

import torch
import torch.nn as nn

from nldpc.decode import KIND_MS, KIND_QMS, KIND_SP, DecodeCfg, decode_autograd, decode_count

from boosted_neural_ldpc_decoder.ConnectingMatrixTorch import ConnectingMatrixTorch
from boosted_neural_ldpc_decoder.Functions import Functions
from boosted_neural_ldpc_decoder.struct.Clipping import Clipping
from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
from boosted_neural_ldpc_decoder.struct.NodeType import NodeType
from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig
from boosted_neural_ldpc_decoder.struct.ParamType import ParamType

_DENSE_BUFFERS = ("W_odd2even", "W_skipconn2even", "W_even2odd", "W_even2odd_with_self", "W_output",
                  "W_skipconn2odd", "Lift_Matrix1", "Lift_Matrix2")
_KIND = {DecoderType.SP: KIND_SP, DecoderType.MS: KIND_MS, DecoderType.QMS: KIND_QMS}


class BoostedNeuralLDPCDecoder(nn.Module):
    def __init__(
            self,
            iter_node_counts,
            batch_size,
            connecting_matrix: ConnectingMatrixTorch,
            node_weight_sharing_config: NodeWeightSharingConfig = NodeWeightSharingConfig(
                cn_weight_sharing=3, ucn_weight_sharing=0, vn_weight_sharing=0),
            decoding_type: DecoderType = DecoderType.QMS,
            decoder_qms_qbit: int = 5,
            fixed_iterative_nodes: list = [],
            fixed_iterative_nodes_init_weight: int = 0,
            allowed_weight_range: Clipping = Clipping(start=0, end=2),
            allowed_bias_range: Clipping = Clipping(start=0, end=2),
            allowed_llr_range: Clipping = Clipping(abs=20.0),
            dtype_cn_weight: torch.dtype = torch.float32,
            dtype_ucn_weight: torch.dtype = torch.float32,
            dtype_vn_weight: torch.dtype = torch.float32,
            init_cn_weight: float = 1,
            init_ucn_weight: float = 1,
            init_vn_weight: float = 1,
            dtype_cn_bias: torch.dtype = torch.float32,
            dtype_ucn_bias: torch.dtype = torch.float32,
            dtype_vn_bias: torch.dtype = torch.float32,
            init_cn_bias: float = 1,
            init_ucn_bias: float = 1,
            init_vn_bias: float = 1,
    ):
        super().__init__()
        self.iter_node_counts = iter_node_counts
        self.batch_size = batch_size
        self.conn_mat = connecting_matrix
        self.N = self.conn_mat.N
        self.M = self.conn_mat.M
        self.Z = self.conn_mat.Z
        self.sum_edge = self.conn_mat.sum_edge
        self.neurons_per_odd_layer = self.conn_mat.neurons_per_odd_layer
        self.neurons_per_even_layer = self.conn_mat.neurons_per_even_layer
        self.node_weight_sharing_config = node_weight_sharing_config
        self.decoding_type = decoding_type
        self.decoder_qms_qbit = decoder_qms_qbit
        self.fixed_iterative_nodes = fixed_iterative_nodes
        self.fixed_iterative_nodes_init_weight = fixed_iterative_nodes_init_weight
        self.allowed_weight_range = allowed_weight_range
        self.allowed_bias_range = allowed_bias_range
        self.allowed_llr_range = allowed_llr_range
        self.dtype_cn_weight, self.dtype_ucn_weight, self.dtype_vn_weight = dtype_cn_weight, dtype_ucn_weight, dtype_vn_weight
        self.init_cn_weight, self.init_ucn_weight, self.init_vn_weight = init_cn_weight, init_ucn_weight, init_vn_weight
        self.dtype_cn_bias, self.dtype_ucn_bias, self.dtype_vn_bias = dtype_cn_bias, dtype_ucn_bias, dtype_vn_bias
        self.init_cn_bias, self.init_ucn_bias, self.init_vn_bias = init_cn_bias, init_ucn_bias, init_vn_bias

        self.outputs = [torch.zeros((self.batch_size, self.N * self.Z), dtype=torch.float32, device=self.conn_mat.device)
                        for _ in range(self.iter_node_counts)]
        self.llr = [None] * (self.iter_node_counts + 1)
        self._register_params()

    # ------------------------------------------------------------------ message state across calls
    class _Pending:
        """The state after `off` iterations of a recorded run (materialised on demand)."""

        def __init__(self, rec, off):
            self.rec, self.off = rec, off

    def _state(self, k):
        """self.llr[k] as a tensor (None = all-zero), recomputing a recorded boundary state."""
        st = self.llr[k]
        if isinstance(st, BoostedNeuralLDPCDecoder._Pending):
            rec, off = st.rec, st.off
            with torch.no_grad():
                state_in = rec["state_in"]
                if state_in is not None and state_in._version != rec["state_ver"]:
                    raise RuntimeError(f"self.llr[{k}] cannot be recomputed: the state its run started from was "
                                       "modified in place after the call that recorded it")
                w = lambda a: None if a is None else a[:off]  # noqa: E731
                cfg = dataclasses.replace(rec["cfg"], keep_state=True)
                _, st = decode_autograd(self.conn_mat.graph, cfg, rec["x"], off, w_cn=w(rec["w_cn"]),
                                        w_ucn=w(rec["w_ucn"]),
                                        w_vn=None if rec["w_vn"] is None else rec["w_vn"][:cfg.vn_prefix + off],
                                        c2v=state_in, app_prev=rec["app_prev"])
            self.llr[k] = st
        return st

    # ------------------------------------------------------------------ parameter registry
    def _param_name(self, param_type: ParamType, node_type: NodeType, iterative_node_identifier: int):
        return f"{param_type.value}_{node_type.value}_{iterative_node_identifier}"

    def _shape_for(self, node_type: NodeType, code: int):
        if code in (1, 4):
            return (int(self.sum_edge),)
        if code in (2, 5):
            return (self.N,) if node_type == NodeType.VN else (self.M,)
        if code == 3:
            return (1,)
        raise ValueError(f"Unsupported sharing type {code} for {node_type}")

    def _iters_with_params(self, code: int):
        if code in (1, 2, 3):
            return list(range(self.iter_node_counts))
        its = [0]
        if self.fixed_iterative_nodes is not None:
            its += list(self.fixed_iterative_nodes)
        return its

    def _register_params(self):
        init = {NodeType.CN: (self.init_cn_weight, self.dtype_cn_weight),
                NodeType.UCN: (self.init_ucn_weight, self.dtype_ucn_weight),
                NodeType.VN: (self.init_vn_weight, self.dtype_vn_weight)}
        for node_type, code in self.node_weight_sharing_config:
            if code == 0:
                continue
            shape = self._shape_for(node_type, code)
            value, dtype = init[node_type]
            for it in self._iters_with_params(code):
                setattr(self, self._param_name(ParamType.Weight, node_type, it),
                        nn.Parameter(torch.full(shape, value, dtype=dtype)))

    def _apply_constraints(self):
        """Clamp weights (and biases, if any exist) into their allowed ranges after a step."""
        for node_type, code in self.node_weight_sharing_config:
            if code == 0:
                continue
            if code in (1, 2, 3):
                its = range(self.iter_node_counts)
            elif self.fixed_iterative_nodes is not None and len(self.fixed_iterative_nodes) > 0:
                its = self.fixed_iterative_nodes
            else:
                its = [0]
            # one multi-tensor clamp per range instead of one kernel per parameter (cfg5: 100 launches a step);
            # clamp_min then clamp_max is clamp_(lo, hi), element for element
            for ptype, rng in ((ParamType.Weight, self.allowed_weight_range),
                               (ParamType.Bias, self.allowed_bias_range)):
                ps = [p.data for p in (getattr(self, self._param_name(ptype, node_type, it), None) for it in its)
                      if p is not None]
                if ps:
                    torch._foreach_clamp_min_(ps, rng.start)
                    torch._foreach_clamp_max_(ps, rng.end)

    def _get_param(self, param_type: ParamType, node_type: NodeType, iterative_node_identifier: int):
        return getattr(self, self._param_name(param_type, node_type, iterative_node_identifier), None)

    def _quantize_message(self, x: torch.Tensor, q_bit: int) -> torch.Tensor:
        return Functions.cal_msa_q_torch(x, q_bit)

    def fetch_param(self, param_type: ParamType, node_type: NodeType, curr_iter: int) -> Optional[torch.Tensor]:
        code = self.node_weight_sharing_config.get(node_type)
        if code in (1, 2, 3):
            return self._get_param(param_type, node_type, curr_iter)
        if code in (4, 5):
            fixed = self.fixed_iterative_nodes
            if fixed and len(fixed) > 0:
                earlier = [i for i in fixed if i <= curr_iter]
                return self._get_param(param_type, node_type, max(earlier) if earlier else fixed[0])
            return self._get_param(param_type, node_type, 0)
        return None

    def get_trainable_parameters(self):
        params = []
        for node_type, code in self.node_weight_sharing_config:
            if code == 0:
                continue
            its = range(self.iter_node_counts) if code in (1, 2, 3) else (self.fixed_iterative_nodes or [0])
            for it in its:
                if it < self.fixed_iterative_nodes_init_weight:
                    continue
                p = self._get_param(ParamType.Weight, node_type, it)
                if p is not None:
                    params.append(p)
        return params

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        for k in _DENSE_BUFFERS:
            state_dict.pop(prefix + k, None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    # ------------------------------------------------------------------ per-iteration weights
    def _per_edge(self, w: torch.Tensor, code: int, what: str) -> torch.Tensor:
        """Expand a CN/UCN weight to one value per C-order edge (differentiable)."""
        E = int(self.sum_edge)
        w = w.to(torch.float32)
        if code == 2:
            return w[self.conn_mat.graph.index_tensor("chk", w.device)]
        if w.numel() == 1:
            return w.reshape(1).expand(E)
        if w.shape[-1] != E or w.numel() != E:
            raise RuntimeError(f"{what}: weight of shape {tuple(w.shape)} does not broadcast against [B, Z, {E}]")
        return w.reshape(E)

    def _per_column(self, w: torch.Tensor, what: str) -> torch.Tensor:
        w = w.to(torch.float32)
        if w.numel() == 1:
            return w.reshape(1).expand(self.N)
        if w.numel() != self.N:
            raise RuntimeError(f"{what}: weight of shape {tuple(w.shape)} does not broadcast against [B, Z, {self.N}]")
        return w.reshape(self.N)

    def _iteration_weights(self, it, fixed_iteration, fixed_iter_weight, fixed_idx, device):
        cfgs = self.node_weight_sharing_config
        cn, ucn, vn = cfgs.get(NodeType.CN), cfgs.get(NodeType.UCN), cfgs.get(NodeType.VN)
        w_vn = None
        if vn in (2, 3):
            w_vn = self._per_column(self.fetch_param(ParamType.Weight, NodeType.VN, it), "VN")
        elif vn == 4:
            wv = fixed_iter_weight[fixed_idx] if it in fixed_iteration else self.fetch_param(ParamType.Weight,
                                                                                              NodeType.VN, it)
            w_vn = self._per_column(torch.as_tensor(wv, device=device), "VN")
        if cn == 0:
            w_cn = None
        elif cn in (1, 2, 3):
            w_cn = self._per_edge(self.fetch_param(ParamType.Weight, NodeType.CN, it), cn, "CN")
        elif cn == 4:
            wc = fixed_iter_weight[fixed_idx] if it in fixed_iteration else self.fetch_param(ParamType.Weight,
                                                                                              NodeType.CN, it)
            w_cn = self._per_edge(torch.as_tensor(wc, device=device), 4, "CN")
        else:
            raise UnboundLocalError("local variable 'x_output_1' referenced before assignment "
                                    f"(CN sharing code {cn} is not handled by the decoder)")
        w_ucn = None
        if ucn > 0 and ucn == cn and cn in (1, 2, 3):
            w_ucn = self._per_edge(self.fetch_param(ParamType.Weight, NodeType.UCN, it), cn, "UCN")
        return w_cn, w_ucn, w_vn

    def _tied(self, node_type):
        """Whether every per-edge weight row repeats one parameter: sharing code 3, one weight per
        iteration (Boosted…py:114-124)."""
        return self.node_weight_sharing_config.get(node_type) == 3

    def _tied_rows(self, node_type, run, width):
        """[len(run), width] rows of one weight each (sharing code 3) as ONE expand of the stacked scalars:
        the same values as stacking the per-iteration expands, but autograd reduces all rows' gradients
        in one kernel instead of one reduction per parameter (cfg5: 100 launches a step)."""
        ps = [self.fetch_param(ParamType.Weight, node_type, t).to(torch.float32).reshape(1) for t in run]
        return torch.stack(ps).expand(len(run), width)

    @torch.no_grad()
    def count_errors(self, xa, y=None, convention=0):
        """Count-only decode (extension): int64 [T, 2] device tensor of (bit errors, frame
        errors) of iterations 0..T-1 of forward(xa) (target_iter None, no fixed iterations), as
        nldpc.channel.ber_counts(outputs, y, convention=...) would count them, without writing the
        posteriors (nor self.outputs / self.llr).  y: [B, N*Z] codeword bits or None (all-zero)."""
        T = self.iter_node_counts
        ws = [self._iteration_weights(it, [], None, 0, xa.device) for it in range(T)]
        stack = lambda k: torch.stack([w[k] for w in ws]) if ws[0][k] is not None else None  # noqa: E731
        w_cn, w_ucn, w_vn = stack(0), stack(1), stack(2)
        qbit = self.decoder_qms_qbit if self.decoding_type == DecoderType.QMS else 0
        cfg = DecodeCfg(kind=_KIND[self.decoding_type], qbit=qbit, ucn=w_ucn is not None,
                        vn_cumulative=w_vn is not None, llr_lo=float(self.allowed_llr_range.start),
                        llr_hi=float(self.allowed_llr_range.end), keep_state=False)
        return decode_count(self.conn_mat.graph, cfg, xa, T, w_cn=w_cn, w_ucn=w_ucn, w_vn=w_vn, y=y,
                            convention=convention)

    # ------------------------------------------------------------------ forward
    def forward(self, xa, target_iter=None, fixed_iter=None, fixed_iter_weight=None):
        """xa: [B, N, Z] tensor (or a per-iteration list); target_iter: None / int / list of
        iterations; fixed_iter / fixed_iter_weight: iterations whose weights are given by the caller.
        Returns self.outputs (target_iter None), one output (int) or a list (list)."""
        if isinstance(target_iter, int):
            iteration = [target_iter]
        elif isinstance(target_iter, list):
            iteration = target_iter  # aliasing kept: fixed_iter entries are appended to the caller's list
        else:
            iteration = list(range(self.iter_node_counts))
        if fixed_iter is not None:
            for each_iter in fixed_iter:
                if each_iter not in iteration:
                    iteration.append(each_iter)
        iteration = sorted(iteration)

        listed = isinstance(xa, list)
        if listed:
            assert len(xa) == len(iteration) - len(fixed_iter)
            assert isinstance(xa[0], torch.Tensor)
        fixed_iteration = []
        if isinstance(fixed_iter, int):
            fixed_iteration = [fixed_iter]
        elif isinstance(fixed_iter, list):
            fixed_iteration = fixed_iter
        if len(fixed_iteration) > 0:
            assert len(fixed_iteration) == len(fixed_iter_weight)

        qbit = self.decoder_qms_qbit if self.decoding_type == DecoderType.QMS else 0
        kind = _KIND[self.decoding_type]
        lo, hi = float(self.allowed_llr_range.start), float(self.allowed_llr_range.end)

        # per-iteration weights (fixed_iter_weight index advances after each fixed iteration)
        device = (xa[0] if listed else xa).device
        weights, fixed_idx = {}, 0
        for it in iteration:
            weights[it] = self._iteration_weights(it, fixed_iteration, fixed_iter_weight, fixed_idx, device)
            if it in fixed_iteration:
                fixed_idx += 1

        # runs of consecutive iterations; a list input or an explicit per-iteration channel
        # restarts the cumulative VN weighting every iteration (reference :321-323)
        runs = []
        for it in iteration:
            if runs and not listed and it == runs[-1][-1] + 1:
                runs[-1].append(it)
            else:
                runs.append([it])
        vn_hist = []  # VN weights already applied to xa_input in this call (cumulative, :329)
        live = {}  # boundary -> state produced by this call (in the autograd graph, as self.llr[t + 1] is)
        for run in runs:
            x_in = xa[run[0]] if listed else xa
            if x_in.dim() != 3 or x_in.shape[0] != self.batch_size:
                raise RuntimeError(f"xa must be [batch_size={self.batch_size}, {self.N}, {self.Z}], "
                                   f"got {tuple(x_in.shape)}")
            w_cn = [weights[t][0] for t in run]
            w_ucn = [weights[t][1] for t in run]
            w_vn = [weights[t][2] for t in run]
            has_vn = w_vn[0] is not None
            prefix = [] if listed else vn_hist
            # a run that ends at the last iteration leaves a state no iteration resumes from (self.llr[T]):
            # the fused kernel does not write it (19.8 GB per cfg3 launch); it stays readable, recomputed
            # on demand like the run's inner boundaries
            last = run[-1] == self.iter_node_counts - 1
            cfg = DecodeCfg(kind=kind, qbit=qbit, ucn=w_ucn[0] is not None, vn_cumulative=has_vn, llr_lo=lo,
                            llr_hi=hi, first_iter=run[0], vn_prefix=len(prefix) if has_vn else 0,
                            keep_state=not last, cn_tied=self._tied(NodeType.CN))
            stack = lambda ws: torch.stack(ws) if ws[0] is not None else None  # noqa: E731
            w_vn_all = torch.stack(prefix + w_vn) if has_vn else None
            if self._tied(NodeType.VN) and has_vn and not prefix:
                w_vn_all = self._tied_rows(NodeType.VN, run, self.N)
            app_prev = None
            if cfg.ucn and run[0] > 0:
                app_prev = self.outputs[run[0] - 1].reshape(self.batch_size, self.N * self.Z).detach()
            # the state this run starts from: this call's own (differentiable) or a stored one (:343, :377)
            state_in = live[run[0]] if run[0] in live else self._state(run[0])
            wc, wu = stack(w_cn), stack(w_ucn)
            if self._tied(NodeType.CN) and wc is not None:
                wc = self._tied_rows(NodeType.CN, run, int(self.sum_edge))
                if wu is not None:
                    wu = self._tied_rows(NodeType.UCN, run, int(self.sum_edge))
            # the entries this run rewrites let go of the previous call's outputs first (the list is refilled
            # below, as the reference's :523 overwrites it): otherwise two T x [B, N*Z] buffers are alive at
            # once (cfg3: 2 x 105 GB); a caller holding those tensors keeps them regardless
            for t in run:
                self.outputs[t] = None
            outs, state = decode_autograd(self.conn_mat.graph, cfg, x_in, len(run), w_cn=wc, w_ucn=wu, w_vn=w_vn_all,
                                          c2v=state_in, app_prev=app_prev)
            for t, o in zip(run, outs):
                self.outputs[t] = o
            dropped = state.numel() == 0  # (the fused path skipped the final state: keep_state=False)
            live[run[-1] + 1] = None if dropped else state
            self.llr[run[-1] + 1] = None if dropped else state
            if len(run) > 1 or dropped:  # boundaries inside the run (and a dropped final state): recomputed on demand
                det = lambda a: None if a is None else a.detach()  # noqa: E731
                # the input and previous posterior are copied (the caller may refill them in place: a
                # 1/T-size copy beside the T outputs); the starting state is module-owned, its version
                # is checked when the record is used
                rec = {"cfg": cfg, "x": x_in.detach().clone(), "w_cn": det(wc), "w_ucn": det(wu),
                       "w_vn": det(w_vn_all), "state_in": det(state_in),
                       "state_ver": None if state_in is None else state_in._version,
                       "app_prev": None if app_prev is None else app_prev.clone()}
                for off in range(1, len(run) + (1 if dropped else 0)):
                    self.llr[run[0] + off] = BoostedNeuralLDPCDecoder._Pending(rec, off)
            if has_vn and not listed:
                vn_hist = vn_hist + w_vn

        if isinstance(target_iter, int):
            return self.outputs[target_iter]
        if isinstance(target_iter, list):
            return [self.outputs[i] for i in target_iter]
        return self.outputs
