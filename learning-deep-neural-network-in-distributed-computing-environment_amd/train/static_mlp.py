"""Static, graph-captured data-parallel training step for MLPs (the flagship path).

The reference's hot loop (BAR/trainer.py:194-223: zero_grad, forward, CE loss,
backward, optimizer.step, three .item() syncs per step) becomes a fixed
schedule of native gfx950 kernels over pre-allocated buffers:

  forward   L x  GEMM + fused bias/activation epilogue          (gemm.hip)
  loss      1 x  fused softmax-xent fwd+bwd+argmax+bias-grad    (xent.hip)
  backward  per layer, WGRAD FIRST: dW_l = dZ_l^T h_{l-1} (fp32, straight into
            the flat grad buffer), then dgrad dZ_{l-1} = (dZ_l W_l) * act'(h_{l-1})
            with the previous layer's bias gradient summed in the same epilogue
  comm      gradient buckets all-reduced on RCCL as soon as their wgrads are
            done -- wgrad-first ordering puts the largest layer's gradient on
            the wire while the remaining dgrad/wgrad GEMMs still run
  optimizer one fused SGD-momentum / Adam launch per bucket, right after that
            bucket's all-reduce lands (overlaps the next bucket's transfer);
            it also refreshes the bf16 weight shadow the GEMMs read

Every stretch of kernels between two collective calls is captured once into a
hipGraph (torch.cuda.CUDAGraph) and replayed, so a step costs a handful of
host calls.  Loss and accuracy accumulate on the device; nothing syncs.

Bucket sizing for xGMI: each MI355X has 7 links (~153 GB/s each);
RCCL spreads a large all-reduce over many channels/links, so buckets are a few
large contiguous ranges (default >= 8 M fp32 elements) rather than 65 per-tensor
messages (BAR/communication.py:4-31).
"""
from __future__ import annotations

import contextlib
import gc
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..ops import _ext
from ..utils.flat_params import FlatParams, storage_numel


@dataclass
class OptimConfig:
    name: str = "sgd"          # "sgd" | "adam" | "adamw"
    lr: float = 0.01
    momentum: float = 0.9
    dampening: float = 0.0
    weight_decay: float = 0.0
    nesterov: bool = False
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8


@contextlib.contextmanager
def no_gc():
    """No Python garbage collection during a graph capture: a collection there can
    destroy an unreachable engine's captured graphs, and destroying a graph exec on
    the capturing thread invalidates the capture (the process aborts)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


class _Segment:
    """A stretch of kernel launches replayed from a captured hipGraph after warmup."""

    def __init__(self, fn, use_graph: bool, warmup: int = 2):
        self.fn, self.use_graph, self.warmup = fn, use_graph, warmup
        self.calls = 0
        self.graph = None

    def __call__(self):
        if not self.use_graph or self.calls < self.warmup:
            self.calls += 1
            self.fn()
            return
        if self.graph is None:
            g = torch.cuda.CUDAGraph()
            # thread_local: other host threads (RCCL / gloo progress, watchdogs) may keep
            # using the HIP runtime while this thread captures
            with no_gc(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.fn()
            self.graph = g
        self.graph.replay()

    @property
    def will_capture(self) -> bool:
        return self.use_graph and self.graph is None and self.calls >= self.warmup


class StaticMLPEngine:
    def __init__(self, model, batch_size: int, optim: OptimConfig | None = None, *, device=None,
                 process_group=None, world_size: int | None = None, bucket_cap_elems: int = 8 << 20,
                 use_graphs: bool = True, average_grads: bool = True, use_head_kernels: bool = True,
                 shard_optimizer: bool | None = None, wgrad_combine: bool = True, library_gemms: bool | None = None,
                 fuse_head_dgrad: bool | None = None, library_dgrad: bool | None = None, head_dgrad_mode: int = -1,
                 relu_masks: bool = True, transposed_dgrad: bool = True, bias_ones_column: bool = True,
                 fuse_head_fwd: bool = True, fuse_head_bwd: bool = True, grad_mix: tuple | None = None,
                 comm_dtype: torch.dtype | None = None):
        """``grad_mix`` = (hops, local_weight): per-step gradient exchange other than the
        equal all-reduce (world > 1) -- hops 0 with a weight = the reference's
        self-weighted all-reduce (BAR/communication.py:4-10), hops 1 / 2 = ring /
        double-ring gossip (BR/communication.py:5-62, BDR/communication.py:5-77), equal
        (local_weight None) or weighted.  Each bucket is exchanged between the backward's
        graph segments (grouped send/recv or all-reduce on RCCL's stream) and combined in
        place by the fused mix kernel (K18) before its optimizer segment.  Every rank
        then applies its OWN mixed gradient (decentralised SGD: replicas differ), so
        these modes run the replicated optimizer.

        ``comm_dtype=torch.bfloat16`` (sharded optimizer, world > 1): the gradient buckets are
        reduce-scattered in bf16 -- (N-1)/N x 2 B per element on xGMI instead of 4.  A plain
        weight-gradient GEMM writes its bf16 output straight into the bf16 staging buffer
        (no cast pass); whatever the wgrads leave in fp32 (split-K slabs, the head's atomics,
        the biases) is cast right before the bucket's collective, and the reduce-scattered
        bf16 shard is widened into the fp32 shard the fused optimizer reads (fp32 master
        weights and optimizer state throughout)."""
        from ..models.mlp import MLP

        if not isinstance(model, MLP):
            raise TypeError("StaticMLPEngine drives ldnn.models.mlp.MLP models")
        self.device = torch.device(device or "cuda")
        if not _ext.use_native(torch.empty(0, device=self.device)):
            raise RuntimeError("StaticMLPEngine needs the native extension on a GPU")
        self.C = _ext.C()
        self.model = model.to(self.device)
        self.B = int(batch_size)
        self.optim = optim or OptimConfig()
        self.pg = process_group
        if world_size is None:
            world_size = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.world = world_size
        self.use_graphs = use_graphs
        self.layers = list(model.layers)
        L = len(self.layers)
        acts = {"none": None, "relu": self.C.EPI_BIAS_RELU, "sigmoid": self.C.EPI_BIAS_SIGMOID}
        self._fwd_epi = [acts[l.activation] if acts[l.activation] is not None else self.C.EPI_BIAS for l in self.layers]
        dacts = {"relu": self.C.EPI_DRELU, "sigmoid": self.C.EPI_DSIGMOID, "none": self.C.EPI_NONE}
        # dgrad of layer l multiplies by the derivative of layer l-1's activation
        self._dgrad_epi = [None] + [dacts[self.layers[l - 1].activation] for l in range(1, L)]
        for l in range(L - 1):
            if self.layers[l].out_features % 8:
                raise ValueError("hidden widths must be multiples of 8")
        if self.layers[0].in_features % 8:
            raise ValueError("input features must be a multiple of 8")

        # flat layout = gradient-ready order: W_L .. W_1, then all biases
        order = [self.layers[l].weight for l in reversed(range(L))] + [l.bias for l in self.layers]
        # ZeRO-1 style sharded optimizer for world > 1: gradients are reduce-SCATTERED
        # (each rank gets 1/N of a bucket), the optimizer updates only that shard, and
        # the new bf16 weights are all-gathered -- 3/4 of an fp32 all-reduce's bytes
        # on xGMI and 1/N of the optimizer's HBM traffic per rank.
        # (shard_optimizer=True also forces the collective path at world 1: a test hook for RCCL)
        if grad_mix is not None and (grad_mix[0] == 0 and grad_mix[1] is None):
            grad_mix = None   # equal all-reduce: the default path
        self._mix_cfg = grad_mix if world_size > 1 else None
        if self._mix_cfg is not None and shard_optimizer:
            raise ValueError("grad_mix modes give every rank its own update: no sharded optimizer")
        if self._mix_cfg is not None:
            shard_optimizer = False
        if comm_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError(f"comm_dtype must be None, torch.float32 or torch.bfloat16, not {comm_dtype}")
        if comm_dtype == torch.bfloat16 and self._mix_cfg is not None:
            raise ValueError("grad_mix modes exchange fp32 gradient buckets (comm_dtype bf16 goes with the "
                             "sharded all-reduce step)")
        self.shard = (self.world > 1) if shard_optimizer is None else bool(shard_optimizer)
        self.distributed = self.world > 1 or self.shard
        # ---- bucket plan: close a bucket after wgrad_l once it holds >= cap elements.
        # Bucket boundaries are padded to a multiple of N x 64 so every bucket splits
        # into N equal, 256-B aligned shards.
        align = self.world * 64 if self.shard else 64
        up = lambda v: (v + align - 1) // align * align  # noqa: E731
        plan, begin, off, align_after = [], 0, 0, {}
        for l in reversed(range(L)):
            off += storage_numel(self.layers[l].weight.shape)
            if l > 0 and self.distributed and off - begin >= bucket_cap_elems:
                align_after[id(self.layers[l].weight)] = align
                off = up(off)
                plan.append(l)
                begin = off
        align_after[id(self.layers[-1].bias)] = align
        self.flat = FlatParams(model, self.device, order=order, align_after=align_after)
        f = self.flat
        self.buckets: list[tuple[int, int, int]] = []   # (begin, end, trigger layer or -1 = end)
        begin = 0
        for l in plan:
            seg = f.seg(self.layers[l].weight)
            end = up(seg.offset + seg.storage_numel)
            self.buckets.append((begin, end, l))
            begin = end
        self.buckets.append((begin, f.numel, -1))
        assert all((e - b) % align == 0 for b, e, _ in self.buckets), self.buckets
        self.W = [f.shadow_storage(l.weight) for l in self.layers]
        self.bias = [f.master_storage(l.bias) for l in self.layers]
        self.dW = [f.grad_storage(l.weight) for l in self.layers]
        self.db = [f.grad_storage(l.bias) for l in self.layers]
        self._bias_begin = f.seg(self.layers[0].bias).offset
        npad = [w.shape[0] for w in self.W]
        self.num_classes = self.layers[-1].out_features

        B, dev, bf = self.B, self.device, torch.bfloat16
        self.x = torch.zeros(B, self.layers[0].in_features, dtype=bf, device=dev)
        self.labels = torch.zeros(B, dtype=torch.long, device=dev)
        self.h = [self.x] + [torch.zeros(B, n, dtype=bf, device=dev) for n in npad]
        self.dz = [None] + [torch.zeros(B, n, dtype=bf, device=dev) for n in npad]
        # classifier head kernels (head.hip): fused last Linear + softmax-xent, and a
        # transposed-read wgrad, for <= 64 (padded) classes
        self.use_head = (npad[-1] % 16 == 0 and npad[-1] <= 64 and self.layers[-1].in_features % 8 == 0
                         and use_head_kernels)
        # fuse_head_dgrad: the head kernel also runs the head's dgrad (dz_{L-1} =
        # dlogits W * act') from its LDS copy of h_{L-1}, instead of a K = 16 GEMM that
        # re-reads h_{L-1}.  Off by default: measured on MI355X at 4096 x 4096 it is
        # not faster (head.hip header)
        # Default (None): on with the library dgrad, where the alternative is a K = 16
        # hipBLASLt GEMM plus the separate dReLU/bias pass over h_{L-1}: measured on
        # MI355X at batch 16384, 1.848 vs 1.887 ms/step.
        # library_gemms: route the plain GEMMs to hipBLASLt (kept as an A/B baseline).
        # Default off: every GEMM of the step runs on ldnn's own MFMA kernels (the
        # four-wave gemm_q.hip for the long-K shapes), with the activation
        # derivative and bias-gradient sums fused into the dgrad epilogue.
        if library_gemms is None:
            library_gemms = False
        if library_dgrad is None:
            library_dgrad = bool(library_gemms)
        if fuse_head_dgrad is None:
            fuse_head_dgrad = True
        # head_dgrad_mode (head.hip): -1 auto = 0 for <= 16 classes (forward-only head
        # kernel + a streaming dh pass with the bias-gradient sums), 1 / 2 = dgrad fused
        # into the head kernel (h re-read from global / staged in LDS)
        self.head_dgrad_mode = int(head_dgrad_mode)
        self.head_dgrad = (bool(fuse_head_dgrad) and self.use_head and L >= 2
                           and (npad[-1] == 16 and self.head_dgrad_mode in (-1, 0, 3)
                                or self.layers[-1].in_features <= self.C.head_dgrad_max_k()))
        # (the streaming head dgrad re-reads h_{L-1} for relu': reading a bit mask written by
        # the previous forward GEMM instead measured ~14 us SLOWER per step at batch 16384 --
        # the GEMM's byte-wise mask stores cost more than the stream saves,
        # profiles/r3/head_dgrad_mask_ab_r3.jsonl)
        self._head_stream = self.head_dgrad and npad[-1] == 16 and self.head_dgrad_mode in (-1, 0)
        # fuse_head_fwd: the last hidden layer's forward GEMM (four-wave kernel,
        # EPI_BIAS_RELU_HEAD) also multiplies each 256-column tile of its ReLU output by
        # the head weight on the MFMA pipe and stores the partial logits; the loss kernel
        # (head_xent_parts) then sums 16 x 64 B per row instead of streaming the 128 MB
        # h_{L-1} again for a K = 4096, N = 16 product (gemm_q.hip head_partial).
        self._head_part = None
        if (fuse_head_fwd and self._head_stream and L >= 2 and self.layers[L - 2].activation == "relu"
                and self.layers[L - 1].in_features % 8 == 0 and npad[-1] == 16):
            self._head_part = torch.empty((self.layers[L - 1].in_features + 255) // 256, B, 16,
                                          dtype=torch.float32, device=dev)
        self._head_db_ws = (torch.empty(self.C.head_dgrad_ws_floats(B, self.layers[-1].in_features),
                                        dtype=torch.float32, device=self.device) if self.head_dgrad else None)
        # [loss_sum, correct] -- one pair per 16-row workgroup of the head kernel
        nslots = (B + 15) // 16 if self.use_head else 1
        self.stats = torch.zeros(nslots, 2, dtype=torch.float32, device=dev)
        self.hp = torch.tensor([self.optim.lr, 0.0], dtype=torch.float32, device=dev)
        o = self.optim
        self.mom = torch.zeros_like(f.master) if (o.name == "sgd" and o.momentum != 0) else None
        if o.name in ("adam", "adamw"):
            self.exp_avg = torch.zeros_like(f.master)
            self.exp_avg_sq = torch.zeros_like(f.master)
        self._grad_scale = 1.0 / self.world if (average_grads and self._mix_cfg is None) else 1.0

        # Gradients produced by accumulation (split-K wgrad atomics, bias-gradient
        # atomics of the xent / dgrad epilogues) must start each step at zero.  The
        # optimizer launch clears them right after consuming them, so the step has
        # no zeroing launch (FlatParams allocates the grads zeroed for step 1).
        #
        # A wgrad whose 128-tile grid leaves CUs idle (e.g. the 4096 x 784 first
        # layer: 224 tiles, one 64-step K loop each) splits its batch reduction and
        # combines the slices IN the launch (gemm.hip k128 + splitk_combine): every
        # CU gets two workgroups, the result is deterministic and overwrites the
        # gradient (no clearing needed).  Tiny grids keep fp32-atomic split-K.
        # library_gemms: the PLAIN GEMMs of the step -- the fp32 weight gradients and
        # the bias(+ReLU) forwards -- go to hipBLASLt (torch.mm out_dtype=fp32 /
        # torch._addmm_activation, both writing into the engine's static buffers);
        # the fused ones stay on ldnn's MFMA kernels: dgrad with the activation
        # derivative and the bias-gradient column sums in its epilogue, and the
        # classifier head (fwd + softmax-xent + argmax, transposed-read wgrad).
        # Measured on MI355X (scripts/bench_blaslt.py, profiles/mlp_gemm_library_r1.jsonl):
        # hipBLASLt is 8-22 % faster on those plain shapes, ldnn wins the fused dgrad.
        hidden = [l for l in range(L) if not (self.use_head and l == L - 1)]
        self._lib_wgrad = [bool(library_gemms) and l in hidden for l in range(L)]
        self._lib_fwd = [bool(library_gemms) and l in hidden and self.layers[l].activation in ("relu", "none")
                         for l in range(L)]
        # library_dgrad: dgrad(l) as a plain hipBLASLt GEMM (bf16 out, in place into dz_l)
        # followed by ONE fused pass (elementwise.hip act_bwd_colsum) that applies layer
        # l-1's activation derivative and emits its bias gradient.  Measured on MI355X
        # (mlp3 784-4096-4096-10, batch 16384, profiles/mlp3_b16384_kernels_r1.txt):
        # ldnn's fused dgrad (dReLU + dbias in the MFMA epilogue) runs the 16384 x 4096
        # x 4096 dgrad at ~0.86 PFLOP/s (639 us) and the K=16 head dgrad in 131 us;
        # hipBLASLt takes 406 + 51 us and the 3-stream pass 2 x 68 us (2.054 -> 1.844
        # ms/step).  Default: on whenever the library GEMMs are.
        # (Splitting the 784-wide wgrad over batch slices with a batched hipBLASLt GEMM
        # was faster in isolation, 160 vs 192 us, scripts/bench_wgrad_split.py, but
        # neutral in the step, so the wgrads stay single GEMMs.)
        self._lib_dgrad = [bool(library_dgrad) and l > 0 and self.layers[l - 1].activation in ("relu", "sigmoid")
                           for l in range(L)]
        self._act_code = [None] + [{"relu": self.C.ACT_RELU, "sigmoid": self.C.ACT_SIGMOID}.get(
            self.layers[l - 1].activation) for l in range(1, L)]
        self.bias_bf16 = [f.shadow_storage(l.bias) for l in self.layers]
        # relu_masks: a ReLU hidden layer's forward (four-wave kernel) also writes a bit
        # mask of its output (1 bit per activation, 1/16 of the bf16 bytes), and the dgrad
        # that needs relu'(h_l) reads the mask instead of h_l -- the dgrad epilogue's
        # 128 MB aux stream at batch 16384 becomes 8 MB (gemm_q.hip EPI_*_MASK).
        self.mask = [None] * (L + 1)
        for l in range(1, L):
            if (relu_masks and self.layers[l - 1].activation == "relu" and not self._lib_fwd[l - 1]
                    and not self._lib_dgrad[l] and not (self.use_head and l == L - 1 and fuse_head_dgrad)):
                self.mask[l] = torch.zeros(B, (npad[l - 1] + 7) // 8, dtype=torch.uint8, device=dev)
        if self._head_part is not None and (self._lib_fwd[L - 2] or self.mask[L - 1] is not None):
            self._head_part = None
        self._db0_from_wgrad = False
        # transposed_dgrad: dgrad(l) reads a transposed bf16 copy of W_l, refreshed by one
        # transpose pass right before it, so both GEMM operands are k-contiguous (measured
        # on MI355X, 16384 x 4096 x 4096: 384-434 vs 430-483 us for the k-strided W)
        self.Wt = [None] * L
        for l in range(1, L):
            if transposed_dgrad and not self._lib_dgrad[l] and not (self.use_head and l == L - 1 and self.head_dgrad):
                self.Wt[l] = torch.zeros(self.W[l].shape[1], self.W[l].shape[0], dtype=bf, device=dev)
        # One transposed copy is written by the fused SGD itself (its bf16 shadow, transposed
        # through LDS per 64 x 64 tile: optim.hip sgd_kernel<TR>) instead of a transpose pass
        # before the dgrad that re-reads the 32 MB shadow: single-process SGD engines (a
        # sharded optimizer updates only its shard; the all-gathered shadow is transposed).
        # The largest eligible matrix takes it; Wt is re-derived whenever the shadow was
        # rewritten outside the step (refresh_shadow / load_state_dict bump its version).
        self._wt_fused = None
        if not self.distributed and self.optim.name == "sgd":
            cand = [l for l in range(1, L) if self.Wt[l] is not None and self.W[l].shape[0] % 64 == 0
                    and self.W[l].shape[1] % 64 == 0 and self.W[l].stride(0) == self.W[l].shape[1]
                    and self.W[l].storage_offset() - f.shadow.storage_offset() == f.seg(self.layers[l].weight).offset]
            if cand:
                self._wt_fused = max(cand, key=lambda l: self.W[l].numel())
        self._wt_ver = None
        self._wgrad_splitk, self._wgrad_ws, self._wgrad_slab = [], [], []
        for l, layer in enumerate(self.layers):
            M, N = self.dW[l].shape
            self._wgrad_ws.append(None)
            self._wgrad_slab.append(None)
            if self.use_head and l == L - 1:
                self._wgrad_splitk.append(self.C.head_wgrad_splits(B, N))
                continue
            if self._lib_wgrad[l]:   # overwrites the gradient: no clearing, no split-K
                self._wgrad_splitk.append(1)
                continue
            t256 = ((M + 255) // 256) * ((N + 255) // 256)
            if B >= 4096 and t256 < 192:
                # long-K wgrad whose 256-tile grid leaves CUs idle (the 4096 x 784 first
                # layer: 64 tiles): the four-wave kernel splits the batch reduction over
                # gridDim.y into separate fp32 slabs and one chip-wide slab_sum adds them
                # (measured on MI355X, 4096 x 784 x 16384: an in-launch combine, where the
                # last-arriving workgroup of a tile re-reads every split's 256 KiB alone,
                # cost ~90 of the kernel's 177 us)
                sk = max(2, min(8, round(256 / t256)))
                Nw = N
                if (l == 0 and bias_ones_column and L >= 2 and self.mask[1] is not None
                        and self.layers[0].bias is not None and (N + 255) // 256 == (N + 8 + 255) // 256):
                    # bias_ones_column: the input buffer carries a ones column after its K0
                    # features, so this wgrad's product has one more column = sum over the
                    # batch of dz_1 = the first layer's bias gradient, in the free part of the
                    # last 256-wide tile; dgrad(1) then needs no bias-gradient sums (measured
                    # on MI355X: the dgrad epilogue's column sums + atomics cost 13-30 us)
                    # (rows padded to a multiple of 64 elements: every row starts on a 128-B line)
                    Nw = N + 8
                    self.xp_full = torch.zeros(B, (Nw + 63) // 64 * 64, dtype=bf, device=dev)
                    self.xp = self.xp_full[:, :Nw]
                    self.xp[:, N] = 1.0
                    self.x = self.xp[:, :N]
                    self.h[0] = self.x
                    self._db0_from_wgrad = True
                self._wgrad_slab[l] = torch.empty(sk, M, Nw, dtype=torch.float32, device=self.device)
                self._wgrad_splitk.append(sk)
                continue
            tile, sk = self.C.gemm_plan(M, N, B, True)
            tiles = ((M + 127) // 128) * ((N + 127) // 128)
            if tile == 128 and wgrad_combine and 64 <= tiles < 256 and B // 64 >= 32:
                sk = max(2, min(4, (2 * 256) // tiles))   # <= 2 workgroups per CU
                ne, nc = self.C.gemm_splitk_ws(M, N, sk)
                self._wgrad_ws[l] = (torch.empty(ne, dtype=torch.float32, device=self.device),
                                     torch.zeros(nc, dtype=torch.int32, device=self.device), 128)
                self._wgrad_splitk.append(sk)
                continue
            self._wgrad_splitk.append(sk if tile == 128 else 1)
        ranges = [(self._bias_begin, f.numel)]
        for l in range(L):
            if self._wgrad_splitk[l] > 1 and self._wgrad_ws[l] is None and self._wgrad_slab[l] is None:  # atomics
                seg = f.seg(self.layers[l].weight)
                ranges.append((seg.offset, seg.offset + seg.storage_numel))
        merged = []
        for b, e in sorted(ranges):
            if merged and b <= merged[-1][1]:
                merged[-1] = (merged[-1][0], max(merged[-1][1], e))
            else:
                merged.append((b, e))
        # the optimizer kernels clear up to two ranges; any further ones get a fill launch.
        # A sharded optimizer never reads the full grad buffer: every range is a fill.
        if self.shard:
            self._opt_zero, self._fill_zero = [], merged
        else:
            self._opt_zero, self._fill_zero = merged[:2], merged[2:]

        if (self._head_part is not None and self.shard
                and self._bucket_of(self.layers[L - 1].weight) != self._bucket_of(self.layers[L - 2].weight)):
            self._head_part = None   # the fused forward would read two buckets' all-gathered weights
        self.rank = dist.get_rank(process_group) if self.distributed else 0
        self._bias_bucket = self._bucket_of(self.layers[0].bias)
        self.xp = getattr(self, "xp", None)
        self._slots = [dict(x=self.x, xp=self.xp, labels=self.labels)]   # slot 0: load_batch's buffers
        self._slot = 0
        self._pending_gather = {}
        self._master_whole = True
        if self.shard:
            self.gshard = [torch.zeros((e - b) // self.world, dtype=torch.float32, device=dev)
                           for b, e, _ in self.buckets]
            self._gloo = dist.get_backend(process_group) == "gloo"
        self.comm_bf16 = comm_dtype == torch.bfloat16 and self.shard
        if self.comm_bf16:
            self._plan_bf16_comm()
        # fuse_head_bwd: the head's dgrad and wgrad in one pass over h_{L-1}, both on the MFMA
        # pipe (head.hip head_bwd; the wgrad accumulates into the gradient the optimizer cleared)
        self._fuse_head_bwd = bool(fuse_head_bwd and self._head_part is not None and L >= 2
                                   and self._dgrad_epi[L - 1] in (self.C.EPI_NONE, self.C.EPI_DRELU)
                                   and self.layers[L - 1].in_features % 64 == 0 and self._wgrad_splitk[L - 1] > 1)
        self._build_segments()
        self._slots[0]["segs"] = (self.segments, self.opt_segments)

    def _plan_bf16_comm(self):
        """bf16 gradient reduce-scatter: the bf16 staging buffer (the flat gradient layout),
        per bucket its bf16 shard, the wgrads that write bf16 directly and, per bucket, the
        fp32 sub-ranges cast right before its collective."""
        f, L, bf, dev = self.flat, len(self.layers), torch.bfloat16, self.device
        self.gbf = torch.zeros(f.numel, dtype=bf, device=dev)
        self.gshard_bf = [torch.zeros((e - b) // self.world, dtype=bf, device=dev) for b, e, _ in self.buckets]
        self.dWb = [None] * L
        for l in range(L):   # plain (unsplit, overwriting) GEMM wgrads: bf16 epilogue, no cast pass
            if (not (self.use_head and l == L - 1) and not self._lib_wgrad[l] and self._wgrad_slab[l] is None
                    and self._wgrad_ws[l] is None and self._wgrad_splitk[l] <= 1):
                d = self.dW[l]
                self.dWb[l] = torch.as_strided(self.gbf, d.shape, d.stride(),
                                               d.storage_offset() - f.grad.storage_offset())
        self._bf16_cast = []
        for b, e, _ in self.buckets:
            direct = sorted((sg.offset, sg.offset + sg.storage_numel)
                            for sg in (f.seg(self.layers[l].weight) for l in range(L) if self.dWb[l] is not None)
                            if b <= sg.offset < e)
            ranges, cur = [], b
            for lo, hi in direct:
                if lo > cur:
                    ranges.append((cur, lo))
                cur = max(cur, hi)
            if cur < e:
                ranges.append((cur, e))
            self._bf16_cast.append(ranges)

    def _cast_bucket(self, bi, whole: bool = False):
        """Stage bucket bi's fp32 gradient ranges into the bf16 buffer (bf16 comm)."""
        b, e, _ = self.buckets[bi]
        for lo, hi in ([(b, e)] if whole else self._bf16_cast[bi]):
            self.C.cast_f32_bf16(self.flat.grad[lo:hi], self.gbf[lo:hi])

    def _widen_shard(self, i):
        self.C.cast_bf16_f32(self.gshard_bf[i], self.gshard[i])

    # ------------------------------------------------------------------ kernels
    def _forward(self, train: bool = False):
        C = self.C
        L = len(self.layers)
        for l in range(L - 1 if (train and self.use_head) else L):
            self._forward_layer(l, train)

    def _loss(self):
        L = len(self.layers)
        if self._head_part is not None:   # logits from the last hidden forward's partial products
            self.C.head_xent_parts(self._head_part, self.bias[L - 1], self.labels, self.h[L], self.dz[L], self.stats,
                                   self.num_classes, 1.0 / self.B)
            if self._fuse_head_bwd:   # + the head's wgrad (dW, db) in the same pass over h
                self.C.head_bwd(self.h[L - 1], self.W[L - 1], self.dz[L], self.dz[L - 1], self.dW[L - 1],
                                self.db[L - 2], self._dgrad_epi[L - 1], self.db[L - 1])
                return
            self.C.head_dgrad_stream(self.h[L - 1], self.W[L - 1], self.dz[L], self.dz[L - 1], self.db[L - 2],
                                     self._dgrad_epi[L - 1])
            return
        if self.use_head:   # last Linear + softmax-xent + argmax (+ the head's dgrad) in one launch
            if self.head_dgrad:
                self.C.head_fwd_xent(self.h[L - 1], self.W[L - 1], self.bias[L - 1], self.labels, self.h[L],
                                     self.dz[L], self.stats, self.num_classes, 1.0 / self.B, dh=self.dz[L - 1],
                                     dbias=self.db[L - 2], dgrad_epi=self._dgrad_epi[L - 1],
                                     dbias_ws=self._head_db_ws, dgrad_mode=self.head_dgrad_mode)
                return
            self.C.head_fwd_xent(self.h[L - 1], self.W[L - 1], self.bias[L - 1], self.labels, self.h[L], self.dz[L],
                                 self.stats, self.num_classes, 1.0 / self.B)
            return
        logits = self.h[L][:, : self.num_classes]
        self.C.softmax_xent(logits, self.labels, self.dz[L][:, : self.num_classes], self.stats,
                            dbias=self.db[L - 1], num_classes=self.num_classes, grad_scale=1.0 / self.B)

    def _wgrad(self, l):
        sk = self._wgrad_splitk[l]
        if self.use_head and l == len(self.layers) - 1:   # also emits the head's bias gradient
            if not self._fuse_head_bwd:   # (else done by head_bwd in _loss)
                self.C.head_wgrad(self.dz[l + 1], self.h[l], self.dW[l], self.db[l], sk)
            return
        if self._lib_wgrad[l]:   # plain GEMM, fp32 out: hipBLASLt straight into the flat grad buffer
            torch.mm(self.dz[l + 1].t(), self.h[l], out_dtype=torch.float32, out=self.dW[l])
            return
        if self._wgrad_slab[l] is not None:   # split-K into slabs + one summing pass, overwrites
            if l == 0 and self._db0_from_wgrad:   # + the ones column: dW_0 and the bias gradient
                self.C.gemm(self.dz[1], self.xp, self._wgrad_slab[0], False, False, tile=256, splitk=sk)
                self.C.slab_sum_cols(self._wgrad_slab[0], self.dW[0], self.db[0])
                return
            self.C.gemm(self.dz[l + 1], self.h[l], self._wgrad_slab[l], False, False, tile=256, splitk=sk)
            self.C.slab_sum(self._wgrad_slab[l], self.dW[l])
            return
        if self._wgrad_ws[l] is not None:   # in-launch split-K combine, overwrites the gradient
            ws, cnt, tile = self._wgrad_ws[l]
            self.C.gemm(self.dz[l + 1], self.h[l], self.dW[l], False, False, tile=tile, splitk=sk, ws=ws, cnt=cnt)
        elif sk > 1:   # accumulates into the grad the previous optimizer launch cleared
            self.C.gemm(self.dz[l + 1], self.h[l], self.dW[l], False, False, beta=1.0, tile=128, splitk=sk)
        elif self.comm_bf16 and self.dWb[l] is not None:   # bf16 comm: straight into the bf16 stage
            self.C.gemm(self.dz[l + 1], self.h[l], self.dWb[l], False, False)
        else:
            self.C.gemm(self.dz[l + 1], self.h[l], self.dW[l], False, False)

    def _dgrad(self, l):
        # dz_l(prev layer output) = (dz_{l+1} W_l) * act'(h_l), bias grad of layer l-1 fused
        if self._lib_dgrad[l]:
            torch.mm(self.dz[l + 1], self.W[l], out=self.dz[l])
            self.C.act_bwd_colsum(self.dz[l], self.h[l], self.dz[l], self.db[l - 1], self._act_code[l], True)
            return
        db = None if (l == 1 and self._db0_from_wgrad) else self.db[l - 1]
        W, w_kc = self.W[l], False
        if self.Wt[l] is not None:
            if l != self._wt_fused:   # (else the previous SGD step wrote it)
                self.C.transpose_bf16(self.W[l], self.Wt[l])
            W, w_kc = self.Wt[l], True
        if self.mask[l] is not None:
            self.C.gemm(self.dz[l + 1], W, self.dz[l], True, w_kc, self.C.EPI_DRELU, dbias=db, mask_in=self.mask[l])
            return
        if w_kc:
            self.C.gemm(self.dz[l + 1], W, self.dz[l], True, True, self._dgrad_epi[l], aux=self.h[l], dbias=db)
            return
        self.C.gemm(self.dz[l + 1], self.W[l], self.dz[l], True, False, self._dgrad_epi[l], aux=self.h[l],
                    dbias=self.db[l - 1])

    def _sync_wt(self):
        """Re-derive the SGD-maintained transposed weight if the shadow was rewritten outside
        the step (first step, refresh_shadow, load_state_dict: an ATen write bumps its version;
        the native kernels' writes do not)."""
        lf = self._wt_fused
        if lf is not None and self._wt_ver != self.flat.shadow._version:
            self.C.transpose_bf16(self.W[lf], self.Wt[lf])
            self._wt_ver = self.flat.shadow._version

    def _shard_range(self, i):
        b, e, _ = self.buckets[i]
        s = (e - b) // self.world
        return b + self.rank * s, b + (self.rank + 1) * s

    def _opt(self, b, e, grad=None, shadow=None):
        f, o, C = self.flat, self.optim, self.C
        p, g = f.master[b:e], (f.grad[b:e] if grad is None else grad)
        sh = f.shadow[b:e] if shadow is None else shadow
        zr = [(max(zb, b) - b, min(ze, e) - b) for zb, ze in self._opt_zero if zb < e and ze > b]
        if o.name == "sgd":
            mom = self.mom[b:e] if self.mom is not None else p
            tk = {}
            lf = self._wt_fused
            if lf is not None and shadow is None:
                off = self.flat.seg(self.layers[lf].weight).offset
                if b <= off and off + self.Wt[lf].numel() <= e:
                    tk = dict(t_begin=off - b, t_out=self.Wt[lf])
            C.sgd_step(p, g, mom, sh, self.hp, self._grad_scale, o.momentum, o.dampening, o.weight_decay,
                       o.nesterov, False, zero_ranges=zr, **tk)
        else:
            C.adam_step(p, g, self.exp_avg[b:e], self.exp_avg_sq[b:e], sh, self.hp, self._grad_scale,
                        o.betas[0], o.betas[1], o.eps, o.weight_decay, o.name == "adamw", zero_ranges=zr)

    # ------------------------------------------------------------ segmentation
    def _build_segments(self):
        L = len(self.layers)
        # backward walk, cut after each bucket's trigger wgrad
        triggers = {t: i for i, (_, _, t) in enumerate(self.buckets) if t >= 0}
        pieces: list[list] = [[]]
        for zb, ze in self._fill_zero:
            pieces[0].append(lambda zb=zb, ze=ze: self.flat.grad[zb:ze].zero_())
        if self.optim.name in ("adam", "adamw"):
            pieces[0].append(lambda: self.C.bump_step(self.hp))
        fwd = lambda: self._forward(train=True)  # noqa: E731
        fwd._ldnn_fwd = True
        pieces[0].append(fwd)
        pieces[0].append(self._loss)
        self._cut_buckets = []
        for l in reversed(range(L)):
            wg = lambda l=l: self._wgrad(l)  # noqa: E731
            wg._ldnn_wgrad = l
            pieces[-1].append(wg)
            if l in triggers:
                if self.comm_bf16:
                    pieces[-1].append(lambda i=triggers[l]: self._cast_bucket(i))
                self._cut_buckets.append(triggers[l])
                pieces.append([])
            if l > 0 and not (self.head_dgrad and l == L - 1):   # (else done by the head kernel)
                pieces[-1].append(lambda l=l: self._dgrad(l))
        self._cut_buckets.append(len(self.buckets) - 1)
        if self.comm_bf16:
            pieces[-1].append(lambda: self._cast_bucket(len(self.buckets) - 1))

        def run(fns):
            def f():
                for fn in fns:
                    fn()
            return f

        if not self.distributed:
            fns = [fn for p in pieces for fn in p] + [lambda: self._opt(0, self.flat.numel)]
            self.segments = [_Segment(run(fns), self.use_graphs)]
            self.opt_segments = []
        elif self.shard:
            self._build_sharded_segments(pieces, run)
        else:
            self.segments = [_Segment(run(p), self.use_graphs) for p in pieces]
            self.opt_segments = [_Segment(run([lambda b=b, e=e: self._opt(b, e)]), self.use_graphs)
                                 for (b, e, _) in self.buckets]

    def _bucket_of(self, t) -> int:
        off = self.flat.seg(t).offset
        for i, (b, e, _) in enumerate(self.buckets):
            if b <= off < e:
                return i
        raise AssertionError("tensor outside every bucket")

    def _build_sharded_segments(self, pieces, run):
        """Sharded step: the forward is cut where the bucket holding the next layer's
        weights changes, so the next step waits for each bucket's weight all-gather
        right before the first kernel that reads it -- the all-gather of the big
        hidden weights overlaps the first layer's GEMM instead of preceding the step.
        (The all-gathers are issued in forward order, see _step_sharded.)"""
        L = len(self.layers)
        n_fwd = L - 1 if self.use_head else L
        p0 = pieces[0]
        i_fwd = next(i for i, fn in enumerate(p0) if getattr(fn, "_ldnn_fwd", False))
        i_loss = next(i for i, fn in enumerate(p0) if fn == self._loss)
        assert i_loss == i_fwd + 1
        prologue, tail = p0[:i_fwd], p0[i_loss + 1:]
        # forward ops in layer order with the bucket each one reads
        ops = [(lambda l=l: self._forward_layer(l, True), self._bucket_of(self.layers[l].weight)) for l in range(n_fwd)]
        ops.append((self._loss, self._bucket_of(self.layers[L - 1].weight)))
        bias_bucket = self._bucket_of(self.layers[0].bias)
        groups, waits = [], []
        for fn, bi in ops:
            if not groups or bi != groups[-1][1]:
                groups.append(([], bi))
                waits.append([bi])
            groups[-1][0].append(fn)
        if bias_bucket not in waits[0]:
            waits[0].insert(0, bias_bucket)
        seg_fns = [list(g) for g, _ in groups]
        seg_fns[0] = prologue + seg_fns[0]
        seg_fns[-1] += tail  # the last forward group runs on into the backward until the first cut
        all_pieces = seg_fns + pieces[1:]
        self._seg_waits = waits + [[] for _ in pieces[1:]]
        self._cut_after = [None] * (len(seg_fns) - 1) + list(self._cut_buckets)
        assert len(self._cut_after) == len(all_pieces)
        self.segments = [_Segment(run(p), self.use_graphs) for p in all_pieces]
        def opt(i):
            if self.comm_bf16:
                self._widen_shard(i)
            self._opt(*self._shard_range(i), grad=self.gshard[i])
        self.opt_segments = [_Segment(run([lambda i=i: opt(i)]), self.use_graphs) for i in range(len(self.buckets))]

    def _forward_layer(self, l, train: bool = False):
        C = self.C
        if train and self._head_part is not None and l == len(self.layers) - 2:
            C.gemm(self.h[l], self.W[l], self.h[l + 1], True, True, C.EPI_BIAS_RELU, bias=self.bias[l],
                   head_w=self.W[l + 1], head_part=self._head_part)
            return
        if self._lib_fwd[l]:
            W = self.W[l]
            if self.layers[l].activation == "relu":
                torch._addmm_activation(self.bias_bf16[l], self.h[l], W.t(), out=self.h[l + 1])
            else:
                torch.addmm(self.bias_bf16[l], self.h[l], W.t(), out=self.h[l + 1])
            return
        if self.mask[l + 1] is not None:
            C.gemm(self.h[l], self.W[l], self.h[l + 1], True, True, C.EPI_BIAS_RELU, bias=self.bias[l],
                   mask_out=self.mask[l + 1])
            return
        C.gemm(self.h[l], self.W[l], self.h[l + 1], True, True, self._fwd_epi[l], bias=self.bias[l])

    # --------------------------------------------------------------------- API
    def set_lr(self, lr: float):
        self.hp[0].fill_(lr)

    def load_batch(self, x: torch.Tensor, y: torch.Tensor):
        self._use_slot(0)
        self.x.copy_(x.reshape(self.B, -1))
        self.labels.copy_(y)

    def add_input_slots(self, n: int) -> list:
        """``n`` more input buffers in the engine's own layout (incl. the first layer's
        ones column), each with its own captured step: a loader (or the benchmark's
        synthetic batches) writes batch i straight into slot i and ``step(slot=i)``
        trains on it -- no per-step copy into a shared input buffer.  Returns the
        [(x [B][in_features] view, labels [B])] of the new slots (ids 1..n)."""
        B, dev, bf = self.B, self.device, torch.bfloat16
        new = []
        for _ in range(int(n)):
            if self.xp is not None:   # ones column after the features (bias_ones_column)
                full = torch.zeros_like(self.xp_full)
                xp = full[:, : self.xp.shape[1]]
                xp[:, self.x.shape[1]] = 1.0
                x = xp[:, : self.x.shape[1]]
            else:
                full, xp, x = None, None, torch.zeros_like(self.x)
            slot = dict(x=x, xp=xp, full=full, labels=torch.zeros_like(self.labels))
            self._slots.append(slot)
            self._use_slot(len(self._slots) - 1, build=True)
            new.append((x, slot["labels"]))
        self._use_slot(0)
        return new

    def _use_slot(self, i: int, build: bool = False):
        if i == self._slot and not build:
            return
        sl = self._slots[i]
        self.x, self.xp, self.labels = sl["x"], sl["xp"], sl["labels"]
        self.h[0] = self.x
        if build:
            self._build_segments()   # closures read self.h[0] / self.xp / self.labels when captured
            sl["segs"] = (self.segments, self.opt_segments)
        self.segments, self.opt_segments = sl["segs"]
        self._slot = i

    def eager_step(self, x: torch.Tensor, y: torch.Tensor):
        """One training step on a batch of ANOTHER size (the trailing partial batch of an
        epoch, BAR/trainer.py:202-216 trains it): the MLP's autograd path on the same
        flat parameters (ldnn native Linear / softmax-xent kernels; its CE adds
        [loss_sum, #correct] into ``stats[0]``), then the engine's fused update.
        Single-process engines only: per-step data parallelism needs the same
        collectives on every rank, so the driver runs the same number of full steps
        everywhere instead."""
        if self.distributed:
            raise RuntimeError("eager_step: a data-parallel engine steps full batches only")
        from ..models.layers import CrossEntropyLoss

        f = self.flat
        self._sync_wt()
        f.grad.zero_()   # the engine's wgrads overwrite: their ranges hold the last step's values
        f._stale.clear()
        with torch.enable_grad():
            self.model.train()
            out = self.model(x.reshape(x.shape[0], -1).to(self.x.dtype))
            loss = CrossEntropyLoss()(out, y, self.stats[0])
            loss.backward()
        if self.optim.name in ("adam", "adamw"):
            self.C.bump_step(self.hp)
        self._opt(0, f.numel)
        return loss.detach()

    def dp_tail_step(self, x: torch.Tensor | None = None, y: torch.Tensor | None = None):
        """Collective (every rank, the same number of times): one data-parallel step on
        batches of ANY size -- the ranks' trailing partial batches, or nothing on a rank
        whose shard ran out (BAR/trainer.py:202-216 trains the short last batch).
        Each rank's gradient is the mean over its own samples (autograd on the flat
        parameters, as eager_step); it is weighted by n_rank * N / n_total before the
        engine's usual collectives, so after the 1/N averaging the update is the mean
        over every rank's samples -- what one process on the concatenated batch does.
        The collectives are a full step's (same buckets, same order), preceded by one
        tiny all-reduce of the sample counts.  Returns the local loss (or None)."""
        if not self.distributed:
            raise RuntimeError("dp_tail_step: single-process engines use eager_step")
        from ..models.layers import CrossEntropyLoss

        n = 0 if y is None else int(y.numel())
        cnt = torch.tensor([float(n)], dtype=torch.float32, device=self.device)
        dist.all_reduce(cnt, group=self.pg)
        n_tot = float(cnt.item())
        if n_tot == 0:
            return None
        self.sync()   # the previous step's weight all-gathers / bias refresh
        self._master_whole = False
        f = self.flat
        f.grad.zero_()
        f._stale.clear()
        if self.optim.name in ("adam", "adamw"):
            self.C.bump_step(self.hp)
        loss = None
        if n > 0:
            with torch.enable_grad():
                self.model.train()
                out = self.model(x.reshape(n, -1).to(self.x.dtype))
                loss = CrossEntropyLoss()(out, y, self.stats[0])
                loss.backward()
            f.finalize_grads()
        if self._mix_cfg is None:   # (gossip / weighted modes: each rank keeps its own gradient's scale)
            f.grad.mul_(n * self.world / n_tot)
        if self.comm_bf16:   # (autograd wrote every gradient in fp32)
            for bi in range(len(self.buckets)):
                self._cast_bucket(bi, whole=True)
        capturing = any(s.will_capture for s in self.opt_segments)
        if self.shard:
            works = []
            for bi in self._cut_buckets:
                w = self._reduce_scatter(bi)
                if capturing and w is not None:
                    w.wait()
                    torch.cuda.current_stream().synchronize()
                works.append((bi, w))
            for bi, w in sorted(works, key=lambda t: -t[0]):
                if w is not None:
                    w.wait()
                self.opt_segments[bi]()
                if bi == self._bias_bucket:
                    self._broadcast_biases(bi, capturing)
                g = self._all_gather(bi)
                if capturing and g is not None:
                    g.wait()
                    torch.cuda.current_stream().synchronize()
                self._pending_gather[bi] = g
        else:
            works = []
            for bi in self._cut_buckets:
                w = self._exchange(bi)
                if capturing:
                    self._wait(w)
                    torch.cuda.current_stream().synchronize()
                works.append((bi, w))
            for bi, w in works:
                self._combine(bi, w)
                self.opt_segments[bi]()
        return None if loss is None else loss.detach()

    # ------------------------------------------------- per-bucket gradient exchange
    def _exchange(self, bi):
        """Start bucket bi's gradient exchange (non-sharded step): the equal / weighted
        all-reduce, or the ring / double-ring neighbour exchange (grad_mix)."""
        b, e, _ = self.buckets[bi]
        g = self.flat.grad[b:e]
        if self._mix_cfg is None:
            return dist.all_reduce(g, group=self.pg, async_op=True)
        hops, w = self._mix_cfg
        bufs = self._mix_bufs(bi)
        if hops == 0:
            bufs[0].copy_(g)   # the own gradient, for the self-weighted mix
            return dist.all_reduce(g, group=self.pg, async_op=True)
        r, N = self.rank, self.world
        sends, recvs = [], []
        for h in range(1, hops + 1):
            src, dst = (r - h) % N, (r + h) % N
            if src == r:   # double ring on 2 ranks: the 2-hop neighbour is this rank
                bufs[h - 1].copy_(g)
                continue
            recvs.append((bufs[h - 1], src))
            sends.append((g, dst))
        if not recvs:
            return None
        glob = (lambda q: q) if self.pg is None else (lambda q: dist.get_global_rank(self.pg, q))
        if self._gloo_backend():
            # gloo: host-staged point-to-point (its device P2P path is slow), synchronous
            from ..parallel.comm import TorchComm

            TorchComm(self.pg).sendrecv(sends, recvs)
            return None
        ops = [dist.P2POp(dist.irecv, t, glob(q), self.pg) for t, q in recvs]
        ops += [dist.P2POp(dist.isend, t, glob(q), self.pg) for t, q in sends]
        return dist.batch_isend_irecv(ops)

    @staticmethod
    def _wait(w):
        for x in (w if isinstance(w, list) else [w]):
            if x is not None:
                x.wait()

    def _combine(self, bi, w):
        """Wait for bucket bi's exchange and mix it in place (fused mix kernel, K18)."""
        self._wait(w)
        if self._mix_cfg is None:
            return
        from ..parallel.aggregation import _mix

        b, e, _ = self.buckets[bi]
        g = self.flat.grad[b:e]
        hops, lw = self._mix_cfg
        bufs = self._mix_bufs(bi)
        N = self.world
        if hops == 0:   # w g + (1-w)(sum - g)/(N-1) = (w - o) g + o sum
            o = (1.0 - lw) / (N - 1)
            _mix(g, bufs[0], g, a=lw - o, b=o)
        elif hops == 1:
            a, c = (0.5, 0.5) if lw is None else (lw, 1.0 - lw)
            _mix(g, g, bufs[0], a=a, b=c)
        else:
            a, c = (1.0 / 3.0, 1.0 / 3.0) if lw is None else (lw, (1.0 - lw) / 2.0)
            _mix(g, g, bufs[0], bufs[1], a=a, b=c, c=c)

    def _mix_bufs(self, bi):
        bufs = self.__dict__.setdefault("_mixb", {})
        if bi not in bufs:
            b, e, _ = self.buckets[bi]
            n = max(1, self._mix_cfg[0])
            bufs[bi] = [torch.empty(e - b, dtype=torch.float32, device=self.device) for _ in range(n)]
        return bufs[bi]

    def _gloo_backend(self) -> bool:
        g = self.__dict__.get("_is_gloo")
        if g is None:
            g = dist.get_backend(self.pg) == "gloo"
            self._is_gloo = g
        return g

    # ------------------------------------------------------------ collectives
    def _rs_buffers(self, i):
        """(input, output) of bucket i's reduce-scatter: bf16 stage / bf16 shard, or fp32."""
        b, e, _ = self.buckets[i]
        if self.comm_bf16:
            return self.gbf[b:e], self.gshard_bf[i]
        return self.flat.grad[b:e], self.gshard[i]

    def _reduce_scatter(self, i):
        src, out = self._rs_buffers(i)
        if self._gloo:   # gloo has no device reduce-scatter: all-reduce, keep this rank's slice
            w = dist.all_reduce(src, group=self.pg, async_op=True)
            w.wait()
            lo, hi = self._shard_range(i)
            b = self.buckets[i][0]
            out.copy_(src[lo - b:hi - b])
            return None
        return dist.reduce_scatter_tensor(out, src, group=self.pg, async_op=True)

    def _all_gather(self, i):
        b, e, _ = self.buckets[i]
        lo, hi = self._shard_range(i)
        if self._gloo:
            out = torch.empty(e - b, dtype=self.flat.shadow.dtype, device=self.device)
            dist.all_gather_into_tensor(out, self.flat.shadow[lo:hi].clone(), group=self.pg)
            self.flat.shadow[b:e].copy_(out)
            return None
        # in place: this rank's shard already sits at its slot of the output
        return dist.all_gather_into_tensor(self.flat.shadow[b:e], self.flat.shadow[lo:hi], group=self.pg,
                                           async_op=True)

    def sync(self):
        """Wait for the previous step's weight all-gathers (the next forward reads them)."""
        for w in self._pending_gather.values():
            if w is not None:
                w.wait()
        self._pending_gather = {}
        self._wait_bias_bcast()

    def _wait_bias_bcast(self):
        for w in getattr(self, "_pending_bias", ()):
            if w is not None:
                w.wait()
        self._pending_bias = []

    def _broadcast_biases(self, bi, capturing):
        """Sharded step: the forward GEMM epilogues and the loss read the fp32 MASTER
        biases, but each rank updates only its shard of the master -- so the owner(s) of
        the bias range send the updated fp32 biases to every rank (a few KB; the
        momentum / Adam state stays with its owner, the only rank that reads it)."""
        b, e, _ = self.buckets[bi]
        sz = (e - b) // self.world
        bb = self._bias_begin
        be = self.flat.seg(self.layers[-1].bias).offset + self.flat.seg(self.layers[-1].bias).storage_numel
        works = []
        for k in range(self.world):
            lo, hi = max(bb, b + k * sz), min(be, b + (k + 1) * sz)
            if lo >= hi:
                continue
            src = k if self.pg is None else dist.get_global_rank(self.pg, k)
            sync = self._gloo or capturing
            w = dist.broadcast(self.flat.master[lo:hi], src=src, group=self.pg, async_op=not sync)
            if sync:
                if capturing:
                    torch.cuda.current_stream().synchronize()
                w = None
            works.append(w)
        self._pending_bias = getattr(self, "_pending_bias", []) + works

    @torch.no_grad()
    def gather_master(self):
        """Make every rank's fp32 master (and optimizer state) whole again after sharded
        steps -- needed before state_dict / checkpoint / evaluation of model.parameters().
        A collective: every rank calls it (a no-op until the next step once done)."""
        if not self.shard or self._master_whole:
            return
        self._master_whole = True
        self.sync()
        bufs = [self.flat.master] + [t for t in (self.mom, getattr(self, "exp_avg", None),
                                                   getattr(self, "exp_avg_sq", None)) if t is not None]
        for i, (b, e, _) in enumerate(self.buckets):
            lo, hi = self._shard_range(i)
            for t in bufs:
                out = torch.empty(e - b, dtype=t.dtype, device=self.device)
                dist.all_gather_into_tensor(out, t[lo:hi].contiguous(), group=self.pg)
                t[b:e].copy_(out)

    def _step_sharded(self, capturing):
        pend = self._pending_gather   # bucket -> the previous step's weight all-gather
        self._pending_gather = {}
        self._wait_bias_bcast()       # the previous step's fp32 bias refresh (the forward reads it)
        works = []
        for i, seg in enumerate(self.segments):
            for bi in self._seg_waits[i]:
                w = pend.pop(bi, None)
                if w is not None:
                    w.wait()
            seg()
            bi = self._cut_after[i]
            if bi is None:
                continue
            w = self._reduce_scatter(bi)
            if capturing and w is not None:
                w.wait()
                torch.cuda.current_stream().synchronize()
            works.append((bi, w))
        for w in pend.values():
            if w is not None:
                w.wait()
        # shard updates in reduce-scatter ISSUE order: the deep buckets (reduced long ago)
        # update while the last bucket's reduce-scatter -- W_0's, fed by the backward's
        # last kernel -- is still on the wire; each update waits only for its own bucket.
        # The weight all-gathers then go out in FORWARD order (the bucket holding W_0 and
        # the biases first): the next step's first GEMM waits only for that one.
        for bi, w in works:
            if w is not None:
                w.wait()
            self.opt_segments[bi]()
            if bi == self._bias_bucket:
                self._broadcast_biases(bi, capturing)
        for bi, _ in sorted(works, key=lambda t: -t[0]):
            g = self._all_gather(bi)
            if capturing and g is not None:
                g.wait()
                torch.cuda.current_stream().synchronize()
            self._pending_gather[bi] = g

    def step(self, slot: int | None = None):
        """One full training step on the batch currently in (self.x, self.labels), or
        in input slot ``slot`` (add_input_slots)."""
        if slot is not None:
            self._use_slot(slot)
        self._master_whole = False
        if not self.distributed:
            self._sync_wt()
            self.segments[0]()
            return
        if self.shard:
            capturing = any(s.will_capture for s in self.segments + self.opt_segments)
            self._step_sharded(capturing)
            return
        # A step that captures a graph runs its collectives synchronously: no
        # collective may be in flight (touching the grad buffers from another
        # stream / thread) while a segment is being captured.
        capturing = any(s.will_capture for s in self.segments + self.opt_segments)
        works = []
        for i, seg in enumerate(self.segments):
            seg()
            bi = self._cut_buckets[i]
            w = self._exchange(bi)
            if capturing:
                self._wait(w)
                torch.cuda.current_stream().synchronize()
            works.append((bi, w))
        for bi, w in works:
            self._combine(bi, w)
            self.opt_segments[bi]()

    def describe(self) -> dict:
        """Which kernel runs each GEMM of the step (bench.py reports it)."""
        L, d = len(self.layers), {}
        for l in range(L):
            if self.use_head and l == L - 1:
                d[f"fwd{l}"] = ("ldnn head_xent_parts (softmax-xent + argmax of the logits the previous forward "
                                "GEMM's epilogue computed on the MFMA pipe)" if self._head_part is not None
                                else "ldnn head_fwd_xent (Linear + softmax-xent + argmax)")
                d[f"wgrad{l}"] = "ldnn head_wgrad"
                if self.head_dgrad:
                    d[f"dgrad{l}"] = ("ldnn head_dgrad_stream (dReLU + bias-gradient sums)" if self._head_stream
                                      else "ldnn head_fwd_xent fused dgrad")
                if self._fuse_head_bwd:
                    d[f"wgrad{l}"] = "ldnn head_bwd (with the dgrad: one pass over h, both on MFMA)"
                    d[f"dgrad{l}"] = "ldnn head_bwd (dReLU + bias-gradient sums, MFMA)"
                continue
            d[f"fwd{l}"] = ("hipBLASLt" if self._lib_fwd[l] else
                            "ldnn gemm_q (bias+ReLU" + (" + ReLU bit mask" if self.mask[l + 1] is not None else "")
                            + (" + head partial logits" if self._head_part is not None and l == L - 2 else "")
                            + " epilogue)")
            if self._lib_wgrad[l]:
                d[f"wgrad{l}"] = "hipBLASLt"
            elif self._wgrad_slab[l] is not None:
                d[f"wgrad{l}"] = (f"ldnn gemm_q split-K x{self._wgrad_splitk[l]} slabs + slab_sum"
                                  + (" (+ bias grad from a ones column)" if l == 0 and self._db0_from_wgrad else ""))
            else:
                d[f"wgrad{l}"] = ("ldnn gemm (auto: gemm_q four-wave 256x256 where gemm_q_preferred, else k256)"
                                  + (f" split-K x{self._wgrad_splitk[l]}" if self._wgrad_splitk[l] > 1 else ""))
            if l > 0:
                d[f"dgrad{l}"] = ("hipBLASLt + act_bwd_colsum" if self._lib_dgrad[l] else
                                  "ldnn gemm_q" + (" on transposed W" if self.Wt[l] is not None else "")
                                  + (" (dReLU from bit mask)" if self.mask[l] is not None else " (fused derivative)"))
        d["optimizer"] = f"ldnn fused {self.optim.name} (flat fp32 master + bf16 shadow)"
        d["library_gemms"] = sum(v.startswith("hipBLASLt") for v in d.values())
        return d

    @torch.no_grad()
    def optimizer_state(self) -> dict:
        """Whole optimizer state (momentum / Adam moments over the flat layout, Adam's
        step count, lr), gathered from the shards first when the optimizer is sharded."""
        self.gather_master()
        st = {"name": self.optim.name, "lr": float(self.hp[0].item()), "step": float(self.hp[1].item()),
              "numel": int(self.flat.numel)}
        for k in ("mom", "exp_avg", "exp_avg_sq"):
            t = getattr(self, k, None)
            if t is not None:
                st[k] = t.detach().cpu().clone()
        return st

    @torch.no_grad()
    def load_optimizer_state(self, st: dict):
        if st.get("name", self.optim.name) != self.optim.name or int(st.get("numel", self.flat.numel)) != self.flat.numel:
            raise ValueError(f"optimizer state of {st.get('name')!r} / {st.get('numel')} elements does not fit "
                             f"this engine ({self.optim.name!r} / {self.flat.numel})")
        for k in ("mom", "exp_avg", "exp_avg_sq"):
            t = getattr(self, k, None)
            if t is not None and st.get(k) is not None:
                t.copy_(st[k].to(t.device))
        self.hp[0].fill_(float(st.get("lr", self.hp[0].item())))
        self.hp[1].fill_(float(st.get("step", 0.0)))

    def reset_stats(self):
        self.stats.zero_()

    def read_stats(self, samples: int):
        self.sync()
        s = self.stats.sum(0).tolist()
        return s[0] / max(samples, 1), 100.0 * s[1] / max(samples, 1)

    @torch.no_grad()
    def predict_logits(self, x: torch.Tensor) -> torch.Tensor:
        self.sync()
        self._use_slot(0)
        self.x.copy_(x.reshape(self.B, -1))
        self._forward()
        return self.h[-1][:, : self.num_classes]
