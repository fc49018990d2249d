"""ResNet-50 v1.5 (the BASELINE.json headline model) on the gfx950 kernel library.

Execution model (MI355X-first):
* activations NHWC bf16; conv filters stored [K, R, S, C] (the implicit-GEMM B operand);
* all variables (conv kernels, BN gamma/beta/moving stats, FC) live in one FlatParams store
  laid out in *backward-completion order*, so gradient all-reduce buckets are contiguous
  slices of the flat gradient buffer that complete front to back during backward;
* every conv+BN(+ReLU)(+residual) unit is hand-scheduled:
    fwd: implicit-GEMM conv whose epilogue emits per-tile BN partial sums -> tiny reduce +
         finalize -> one fused apply pass (scale/shift, residual add, ReLU);
    bwd: one fused BN-backward reduce pass (ReLU mask from the saved output, shortcut
         gradient emitted on the fly) -> finalize -> apply -> wgrad (split-K, fp32 straight
         into the flat gradient slice) + dgrad (accumulating into the shortcut gradient);
* the explicit forward/backward order gives the collective engine exact "gradient ready"
  points, and makes the whole step capturable into hipGraphs.

Variable names follow tf.keras.applications.ResNet50 (conv{stage}_block{b}_{i}_conv/kernel,
..._bn/{gamma,beta,moving_mean,moving_variance}, predictions/{kernel,bias}); checkpoint
conversion to TF's [R,S,C,K] kernel layout happens in the checkpoint layer.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ..train.flat import FlatParams, ParamSpec
from ..utils import graphs

STAGES_50 = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))


def _he_init(fan_in):
    std = math.sqrt(2.0 / fan_in) / 0.87962566103423978  # truncated-normal (+-2 sigma) correction

    def init(t, gen):
        t.normal_(0.0, std, generator=gen)
        t.clamp_(-2 * std, 2 * std)
    init.dev = (1, 0.0, std)  # device init: truncated normal (init.hip)
    return init


def _fill(v):
    def init(t, gen):
        t.fill_(v)
    init.dev = (3, float(v), 0.0)
    return init


def _glorot(fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))

    def init(t, gen):
        t.uniform_(-lim, lim, generator=gen)
    init.dev = (2, -lim, lim)
    return init


@dataclass
class ConvSpec:
    name: str
    cin: int
    cout: int
    k: int
    stride: int
    pad: int
    cin_store: int  # channels as stored (stem input padded 3 -> 8)


class ResNet:
    """precision="fp8" (BASELINE.json config 5): every conv whose input has a multiple of 128
    channels runs its forward GEMM in fp8 e4m3 on the block-scaled MFMA
    (ops.gemm.conv_fwd_fp8): the producing BN-apply pass writes an fp8 copy of its output
    with a delayed per-tensor scale (device-side amax history, ops/fp8.hip), the conv weights
    are re-quantised once per step with current per-tensor scaling, and the dequantisation
    scales reach the GEMM epilogue as device pointers (no host sync, graph-capturable).
    Backward (dgrad/wgrad) stays bf16 on the same saved bf16 activations."""

    def __init__(self, stages=STAGES_50, num_classes=1000, in_channels=3, device="cuda", seed=0,
                 bn_momentum=0.9, bn_eps=1e-5, width=64, precision="bf16"):
        if precision not in ("bf16", "fp8"):
            raise ValueError("precision must be bf16 or fp8")
        self.precision = precision
        # dgrad epilogues emit the next BN-backward's masked gradient + partial sums
        # (TTD_FUSE_BN_BWD=0 restores the separate statistics pass, for A/B runs)
        self.fuse_bn_bwd = os.environ.get("TTD_FUSE_BN_BWD", "1") != "0"
        self.device = torch.device(device)
        # weight gradients on a second HIP stream (TTD_WGRAD_STREAM=0: single stream)
        self.wgrad_stream = os.environ.get("TTD_WGRAD_STREAM", "1") != "0" and self.device.type == "cuda"
        # projection-shortcut backward (BN backward + strided dgrad) on the side stream, concurrent
        # with the block's c3 -> c2 data-gradient chain (joins before c1's dgrad accumulates into it)
        self.cd_side = os.environ.get("TTD_CD_SIDE", "1") != "0"
        # forward projection shortcut on the side stream, concurrent with the block's c1 -> c2
        # (TTD_FWD_PROJ_SIDE=0: inline on the main stream — no fork / join, fewer graph segments)
        self.fwd_proj_side = os.environ.get("TTD_FWD_PROJ_SIDE", "1") != "0"
        # ... joined after the block's c3 when c3's BN apply is deferred into the next c1
        # (TTD_LATE_PROJ_JOIN=0: before c3, as the apply pass needs it)
        self.late_proj_join = os.environ.get("TTD_LATE_PROJ_JOIN", "1") != "0"
        # precision="fp8": unit-stride 3x3 data gradients on the fp8 MFMA with e5m2 gradients
        # (TTD_FP8_DGRAD=0: bf16 data gradients)
        self.fp8_dgrad = os.environ.get("TTD_FP8_DGRAD", "1") != "0"
        # fp8 weight gradients of the convs that have both fp8 copies already (the e4m3 input of the
        # fp8 forward and the e5m2 dz of the fp8 data gradient): ops.gemm.conv_wgrad_fp8
        self.fp8_wgrad = os.environ.get("TTD_FP8_WGRAD", "1") != "0"
        self.fp8_only_input = os.environ.get("TTD_FP8_ONLY_INPUT", "1") != "0"
        # precision="fp8": the 1x1 convs with >= 128 input and output channels on fp8 too — forward
        # from the e4m3 copy the producing BN apply writes, unit-stride data gradients from the e5m2
        # dz the BN backward-apply pass writes (with the shortcut-gradient accumulate and the
        # feeding BN's statistics in the epilogue), weight gradients from both copies
        # (TTD_FP8_1X1=0: 3x3 convs only, the 1x1 convs keep their fused bf16 kernels)
        self.fp8_1x1 = os.environ.get("TTD_FP8_1X1", "1") != "0"
        # ... and their weight gradients from the fp8 copies (TTD_FP8_1X1_WGRAD=0: bf16 weight
        # gradients on the 4-wave transposed-read kernel; the bf16 input and dz stay stored)
        self.fp8_1x1_wgrad = os.environ.get("TTD_FP8_1X1_WGRAD", "1") != "0"
        # ... the strided 1x1 projection shortcuts' forward too (TTD_FP8_1X1_S2=1; their data
        # gradient is bf16 either way: the fp8 one has no sampled-pixel form)
        self.fp8_1x1_s2 = os.environ.get("TTD_FP8_1X1_S2", "0") != "0"
        self._x8 = {}
        self._x_unstored = set()
        # projection-shortcut BN applied inside the block's last BN pass (its normalised output is
        # never stored: two HBM passes of the stage's largest tensor saved; TTD_FUSE_PROJ=0: off)
        self.fuse_proj = os.environ.get("TTD_FUSE_PROJ", "1") != "0"
        # stride-2 projection dgrad without the zero fill of its output (TTD_SAMPLED_DGRAD=0: A/B)
        self.sampled_dgrad = os.environ.get("TTD_SAMPLED_DGRAD", "1") != "0"
        # streaming pointwise kernel (ops.gemm.pw_conv) with the neighbouring BN pass fused in as its
        # operand prologue, on the shapes where it measured faster (tools/pw_bench.py); TTD_FUSE_PW=0: off
        # (fp8 runs them too: only the 3x3 convs with >= 128 input channels take fp8 operands, and
        # none of the fused producer / consumer pairs below is one of those)
        self.fuse_pw = os.environ.get("TTD_FUSE_PW", "1") != "0"
        # individual switches (A/B and debugging): plain pw forward, c2->c3, c3->next c1, dgrad
        self.pw_parts = {"plain": True, "c23": True, "c31": True, "dgrad": True}
        # halo-tiled 3x3 kernel (ops.gemm.conv3_halo) for the shapes it is compiled for, with the
        # producing BN apply / BN backward fused in as its operand prologue; TTD_FUSE_C3=0: off
        self.fuse_c3 = os.environ.get("TTD_FUSE_C3", "1") != "0"
        # halo-kernel data gradient of those convs: 2 = after the BN-backward pass, with the feeding
        # unit's BN-backward sums in its epilogue (tools/conv3_bench.py: 648 -> 529 us at b1024);
        # 1 = with the BN backward as its operand prologue (slower: 920 vs 863 us incl. the pass)
        self.c3_dgrad = int(os.environ.get("TTD_C3_DGRAD", "2"))
        # 1x1 data gradients on the 256-row kernel form the unit's BN backward (dz = a*g + b*y + c)
        # in LDS as their operand and store dz for the weight gradient: no separate backward-apply
        # pass, no re-read of dz (ops.gemm.conv_dgrad(bn_pro=...)); TTD_DGRAD_BNPRO=0: off
        self.bn_pro = os.environ.get("TTD_DGRAD_BNPRO", "1") != "0"
        # the block output h = relu(bn3(y3) + shortcut) formed inside the next block's c1 conv
        # (256-row kernel operand prologue, stores h + ReLU bits): no BN apply pass for the
        # stage-3/4 blocks the streaming pointwise kernel does not take; TTD_FWD_BNPRO=0: off
        self.fwd_pro = os.environ.get("TTD_FWD_BNPRO", "1") != "0"
        # the streaming-kernel data gradients with the BN-backward prologue (stage-2 c1 / c3) also
        # form their conv's weight gradient from the dz tile in LDS (pw_gemm.hip WG); 0: separate
        # side-stream weight-gradient pass over a stored dz
        self.pw_wgrad = os.environ.get("TTD_PW_WGRAD", "1") != "0"
        self.pw_fold_side = os.environ.get("TTD_PW_FOLD_SIDE", "1") != "0"
        # cap on the persistent workgroups of that kernel when it runs on the side stream (the
        # stage-2 projection; 0 = one per CU). It holds every CU while it runs, but the main chain
        # joins on it right after: 128 / 64 measured 0.3 / 2.1 ms slower per step than the full grid
        self.side_pw_wgs = int(os.environ.get("TTD_SIDE_PW_WGS", "0"))
        # stem weight gradient on its dedicated kernel (3 real input channels, BN backward on the fly)
        self.stem_kernel = os.environ.get("TTD_STEM_WGRAD", "1") != "0"
        # dedicated stem forward kernel (stem_fwd.hip: K = 7 x 32 over the 3 real channels)
        self.stem_fwd_kernel = os.environ.get("TTD_STEM_FWD", "1") != "0"
        self._wgrad_stream = None
        # every data-gradient filter operand prepared in one launch per step (TTD_WPREP=0: per conv)
        self.wprep = os.environ.get("TTD_WPREP", "1") != "0"
        self._wp_cur = None
        self.num_classes = num_classes
        self.in_channels = in_channels
        self.in_store = 8 if in_channels <= 8 else (in_channels + 7) // 8 * 8
        self.bn_momentum = bn_momentum
        self.bn_eps = bn_eps
        self.stem = ConvSpec("conv1", in_channels, width, 7, 2, 3, self.in_store)
        self.blocks = []  # list of dicts
        cin = width
        for si, (mid, n, stride) in enumerate(stages):
            for b in range(n):
                s = stride if b == 0 else 1
                pre = "conv%d_block%d" % (si + 2, b + 1)
                blk = {
                    "c1": ConvSpec(pre + "_1", cin, mid, 1, 1, 0, cin),
                    "c2": ConvSpec(pre + "_2", mid, mid, 3, s, 1, mid),
                    "c3": ConvSpec(pre + "_3", mid, mid * 4, 1, 1, 0, mid),
                    "cd": ConvSpec(pre + "_0", cin, mid * 4, 1, s, 0, cin) if (s != 1 or cin != mid * 4) else None,
                }
                self.blocks.append(blk)
                cin = mid * 4
        self.feat = cin
        self.params = FlatParams(self._specs(), self.device, seed=seed,
                                 device_init=os.environ.get("TTD_DEVICE_INIT", "1") != "0")
        self._fp8 = None
        if precision == "fp8" and self.device.type == "cuda":
            self._init_fp8()

    # ----------------------------------------------------------------- fp8 state
    def _fp8_conv(self, c: ConvSpec) -> bool:
        # fp8 where it pays end to end: the 3x3 convs (compute-bound: fp8 MFMA at 2x the bf16
        # rate, 15-43 % faster at the b1024 shapes, tools/fp8_conv_ab.py), K in 128-element
        # tiles, >= 128 output channels. The 1x1 convs are store-bound (5-23 % faster alone);
        # forward-only fp8 there (the producing BN pass writing an fp8 copy next to the bf16 one)
        # measured 1 % slower per step, so with fp8_1x1 they also take the fp8 data and weight
        # gradients and the bf16 input copy is dropped where nothing else reads it.
        if self.precision != "fp8" or c.cin_store % 128 or c.cout < 128:
            return False
        return c.k > 1 or (self.fp8_1x1 and c.k == 1 and (c.stride == 1 or self.fp8_1x1_s2))

    def _init_fp8(self):
        P = self.params
        convs = [c for c in self.conv_list() if self._fp8_conv(c)]
        rows = []
        self._w8_slot = {}
        for i, c in enumerate(convs):
            name = c.name + "_conv/kernel"
            rows.append((P.offsets[name], int(np.prod(P.spec(name).shape)), i))
            self._w8_slot[c.name] = i
        arr = np.zeros(len(rows), dtype=np.dtype([("off", "<i8"), ("len", "<i4"), ("slot", "<i4")]))
        for i, r in enumerate(rows):
            arr[i] = r
        self._w8_table = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)
        self._w8_n = len(rows)
        self._w8_max = max(r[1] for r in rows)
        self._w8_flat = torch.zeros(P.numel, dtype=torch.uint8, device=self.device)
        from ..ops.kernels import FP8_SLOT
        self._w8_slots = torch.zeros((len(rows), FP8_SLOT), dtype=torch.float32, device=self.device)
        self._w8 = {c.name: self._w8_flat[P.offsets[c.name + "_conv/kernel"]:P.offsets[c.name + "_conv/kernel"]
                                          + int(np.prod(P.spec(c.name + "_conv/kernel").shape))]
                    .view(P.spec(c.name + "_conv/kernel").shape) for c in convs}
        # activation slots: one per fp8-consumed tensor, assigned in forward order
        self._a_slots = torch.zeros((4 * len(self.blocks) + 4, FP8_SLOT), dtype=torch.float32, device=self.device)
        self._a_slots[:, 2] = 1.0
        self._a_slots[:, 3] = 1.0
        # fp8 data gradients (unit-stride 3x3 convs with >= 128 output channels: the stage 3-5 c2
        # units off the halo kernel): dz in OCP e5m2 with delayed per-tensor scaling (one slot per
        # conv; the BN backward-apply pass that produces dz writes the copy and this step's amax),
        # the filter transposed to [C,R,S,K] in e4m3 with current scaling (from the step's
        # WeightPrep buffer). The first step only collects the gradient amax (bf16 dgrad).
        self._g8 = {c.name: i for i, c in enumerate(c for c in self.conv_list() if self._fp8_dgrad_conv(c))}
        # e5m2 dz slots: the fp8-dgrad convs first (their row index is shared with the transposed
        # e4m3 filter table), then the convs whose weight gradient alone runs on fp8 (the strided
        # 3x3 convs with an fp8 forward: bf16 sub-pixel data gradient, fp8 weight gradient)
        self._gq = dict(self._g8)
        for c in self.conv_list():
            if c.name not in self._gq and self._fp8_conv(c) and c.k > 1 and c.stride > 1:
                self._gq[c.name] = len(self._gq)
        self._g_slots = torch.zeros((max(1, len(self._gq)), FP8_SLOT), dtype=torch.float32, device=self.device)
        self._g_slots[:, 2] = 1.0
        self._g_slots[:, 3] = 1.0
        self._fp8_bwd_steps = 0
        self._fp8 = True

    def _fp8_dgrad_conv(self, c: ConvSpec) -> bool:
        if not (self.precision == "fp8" and self.fp8_dgrad and c.stride == 1 and c.cout % 128 == 0):
            return False
        if c.k == 1:
            # (not a c3 whose forward runs bf16 on the streaming kernel with c2's BN apply fused:
            # no e4m3 input for an fp8 weight gradient, and its fused BN-backward dgrad is cheaper)
            return self._fp8_conv(c) and not (self._pw_part("c23") and self._pw_fwd_ok(c, True))
        return c.k == 3 and c.cin_store % 8 == 0 and not self._c3_ok(c, 56, 56)

    def _g8_take(self, c: ConvSpec, need_dx, feeds, feeds2, dx, dx_beta, dx_sampled) -> bool:
        """This backward of c goes through the e5m2 dz copy (ops.gemm.conv_dgrad_fp8 from the
        second step on; the first step's pass only collects the gradient amax), so the bf16 fused
        data-gradient kernels (BN-backward operand prologue, streaming pointwise) are bypassed.
        The fp8 data gradient has the feeding-BN epilogue (one fed unit) and a dense beta
        accumulate, not the sampled-pixel one of a strided projection's gradient."""
        return (self._fp8 is not None and need_dx and c.name in self._g8 and self._wp_cur is not None
                and feeds is not None and feeds2 is None and (dx is None or bool(dx_beta)) and not dx_sampled)

    def _fp8_step_begin(self):
        from ..ops import kernels as K
        K.fp8_rollover(self._a_slots, margin=0.9)
        if self._gq:
            K.fp8_rollover(self._g_slots, margin=0.5, fmax=57344.0)
        K.fp8_quant_weights(self.params.compute, self._w8_flat, self._w8_table, self._w8_n, self._w8_max,
                            self._w8_slots)
        self._a_next = 0

    def _new_a_slot(self):
        i = self._a_next
        self._a_next += 1
        return self._a_slots[i]

    # ----------------------------------------------------------------- variables
    def _conv_specs(self, c: ConvSpec):
        fan_in = c.k * c.k * c.cin
        return [
            ParamSpec(c.name + "_conv/kernel", (c.cout, c.k, c.k, c.cin_store), _he_init(fan_in), True,
                      meta={"layout": "KRSC", "tf_shape": (c.k, c.k, c.cin, c.cout), "cin": c.cin}),
            ParamSpec(c.name + "_bn/gamma", (c.cout,), _fill(1.0), False),
            ParamSpec(c.name + "_bn/beta", (c.cout,), _fill(0.0), False),
            ParamSpec(c.name + "_bn/moving_mean", (c.cout,), _fill(0.0), False, trainable=False),
            ParamSpec(c.name + "_bn/moving_variance", (c.cout,), _fill(1.0), False, trainable=False),
        ]

    def _specs(self):
        specs = [
            ParamSpec("predictions/kernel", (self.feat, self.num_classes), _glorot(self.feat, self.num_classes), True),
            ParamSpec("predictions/bias", (self.num_classes,), _fill(0.0), False),
        ]
        for blk in reversed(self.blocks):  # backward-completion order
            for key in ("c3", "c2", "cd", "c1"):
                if blk[key] is not None:
                    specs += self._conv_specs(blk[key])
        specs += self._conv_specs(self.stem)
        # zero the padded input channels of the stem kernel (they must stay zero)
        stem_k = specs[-5]
        base_init = stem_k.init
        cin = self.in_channels

        def stem_init(t, gen, base_init=base_init, cin=cin):
            base_init(t, gen)
            t[..., cin:] = 0.0
        stem_k.init = stem_init
        return specs

    def conv_list(self) -> List[ConvSpec]:
        out = [self.stem]
        for blk in self.blocks:
            out += [blk[k] for k in ("c1", "c2", "c3", "cd") if blk[k] is not None]
        return out

    # ----------------------------------------------------------------- GPU engine
    def _pw_fwd_ok(self, c: ConvSpec, fused_input: bool) -> bool:
        """Forward 1x1 conv on the streaming kernel: K <= 128 (wide output, short reduction), or
        K = 256 when it also absorbs the producer's BN apply (tools/pw_bench.py A/B, b1024)."""
        from ..ops import gemm as G
        if not (self.fuse_pw and self.device.type == "cuda" and c.k == 1 and c.stride == 1 and c.pad == 0):
            return False
        if not G.pw_ok(1 << 20, c.cout, c.cin_store):
            return False
        return c.cin_store <= 128 or (fused_input and c.cin_store == 256)

    def _pw_part(self, name):
        return self.fuse_pw and self.pw_parts.get(name, True)

    # (dz channels, dx channels) of the data gradients that run faster on the streaming kernel with
    # the unit's BN backward as prologue and the LDS-DMA epilogue (tools/pw_bench.py, b1024):
    # stage-2 c3 (256 -> 64) and c1 (64 -> 256, accumulating into the shortcut gradient)
    # (the stage-3 c1s, 128 -> 256 / 512, measured slower there: 66.7 / 67.7 vs 65.9 ms per step)
    PW_DGRAD_SHAPES = {(256, 64), (64, 256)}

    # 1x1 dgrads with the BN backward as LDS operand prologue where it measured faster than the
    # backward-apply pass + plain dgrad (tools/dgrad_bnpro_bench.py, b1024,
    # profiles/r3_dgrad_bnpro_ab_b1024.txt): stage-3/4 c3 (dz 512 / 1024 ch -> 128 / 256: 1.30x /
    # 1.06x) and the stage-3 c1s (-> 256 / 512 ch: 1.08x / 1.03x). Wider outputs recompute the
    # operand per column tile (stage-4/5 c1: 0.88x / 0.81x) and 32-K-tile loops lose the
    # ping-pong schedule (stage-5 c3: 0.81x): those keep the pass.
    BNPRO_MAX_K = 1024
    BNPRO_MAX_N = 512
    # forward apply prologue (h = relu(bn3(y3) + shortcut) formed in the next c1's operand tile):
    # faster at the stage-3 widths (512 -> 128: 1.18x, 512 -> 256: 1.04x), slower at stage 4
    # (1024 -> 256: 0.90x, with the projection BN 0.87x): tools/dgrad_bnpro_bench.py --fwd
    FWDPRO_MAX_K = 512

    def _fwd_pro_ok(self, c: ConvSpec, x_shape) -> bool:
        """c (a 1x1 unit-stride conv) takes its input's BN apply + residual + ReLU as the 256-row
        kernel's operand prologue (ops.gemm.conv_fwd_bnpro)."""
        from ..ops import gemm as G
        return (self.fwd_pro and self.device.type == "cuda" and c.k == 1 and c.stride == 1 and c.pad == 0
                and c.cin_store <= self.FWDPRO_MAX_K and c.cout <= self.BNPRO_MAX_N and not self._fp8_conv(c)
                and G.conv_fwd_bnpro_ok(tuple(x_shape), (c.cout, 1, 1, c.cin_store)))

    def _pw_dgrad_ok(self, c: ConvSpec) -> bool:
        from ..ops import gemm as G
        return (self.fuse_pw and self.device.type == "cuda" and c.k == 1 and c.stride == 1 and c.pad == 0
                and (c.cout, c.cin_store) in self.PW_DGRAD_SHAPES and G.pw_ok(1 << 20, c.cin_store, c.cout))

    def _stem_packed_ok(self, shape) -> bool:
        """Both stem kernels (stem_fwd.hip, stem_wgrad.hip) take the unpadded [N,H,W,3] images."""
        from ..ops import gemm as G
        c = self.stem
        w = (c.cout, c.k, c.k, c.cin_store)
        from ..ops import kernels as K
        return (self.device.type == "cuda" and self.stem_fwd_kernel and self.stem_kernel and self.fuse_bn_bwd
                and shape[-1] == self.in_channels and K.stem_pool_fusable((shape[0], 112, 112, c.cout))
                and G.stem_fwd_ok(shape, w, (c.stride, c.stride), (c.pad, c.pad), self.in_channels)
                and G.stem_wgrad_ok(shape, w, (c.stride, c.stride), (c.pad, c.pad), self.in_channels))

    def _c3_ok(self, c: ConvSpec, H: int, W: int) -> bool:
        """3x3/s1 conv on the halo kernel (its input is H x W)."""
        from ..ops import gemm as G
        return (self.fuse_c3 and self.device.type == "cuda" and c.k == 3 and c.stride == 1 and c.pad == 1
                and G.conv3_rows(H, W, c.cin_store, c.cout) > 0)

    def _convbn_fwd(self, c: ConvSpec, x, relu, residual=None, x8=None, want8=False, pool=False, defer=False,
                    residual_bn=None, pro=None, pro_big=False, store_out=True):
        """conv + BN (+residual) (+ReLU). x8 = (fp8 copy of x, its scale slot) selects the fp8
        forward GEMM; want8 makes the BN-apply pass also emit an fp8 copy of the output.
        defer=True: no apply pass — returns the raw conv output (the consumer applies this BN
        through residual_bn = (scale, shift) of its own apply pass).
        pool=True (stem): BN + ReLU + 3x3/s2 max pooling in one pass that never stores the
        BN+ReLU output; returns (pooled, ctx, argmax).
        pro=(scale, shift, res, res_bn, side, side_mask): x is the RAW conv output of the producing
        unit; its BN apply (+ residual) runs inside this conv's operand load (streaming pointwise
        kernel, or pro_big: the 256-row kernel's operand prologue) and the applied tensor / its ReLU
        bits land in side / side_mask (this unit's input).
        Returns (out, ctx) or (out, ctx, out8) when want8."""
        from ..ops import gemm as G
        from ..ops import kernels as K
        P = self.params
        N, H, W, C = x.shape
        Pp = (H + 2 * c.pad - c.k) // c.stride + 1
        Q = (W + 2 * c.pad - c.k) // c.stride + 1
        M = N * Pp * Q
        bm = 128 if M > 64 else 64
        bn = 128 if c.cout > 64 else 64
        big = G.big_bn(M, c.cout, c.k * c.k * c.cin_store)
        use8 = x8 is not None and self._fp8_conv(c)
        if use8:
            bm, bn = 256, (256 if c.cout >= 256 else 128)
        elif big and c.cin_store % 64 == 0:
            bm, bn = 256, big  # 256-row LDS-DMA kernel (BN stat rows per 256-pixel tile)
        T = -(-M // bm)
        partial = None
        if (c is self.stem and not use8 and self.stem_fwd_kernel and self.device.type == "cuda"
                and G.stem_fwd_ok(tuple(x.shape), tuple(P.var[c.name + "_conv/kernel"].shape), (c.stride, c.stride),
                                  (c.pad, c.pad), self.in_channels)):
            y, partial, T = G.stem_fwd(x, P.c[c.name + "_conv/kernel"])
        elif not use8 and self._c3_ok(c, H, W):
            w4 = P.c[c.name + "_conv/kernel"]
            if pro is not None:
                psc, psh, _, _, side, side_mask = pro
                y, partial, T = G.conv3_halo(x, w4, prologue=("bn_fwd", psc, psh, side, side_mask), stat=True)
                x = side  # the unit's input as the backward needs it
            else:
                y, partial, T = G.conv3_halo(x, w4, stat=True)
        elif pro is not None and pro_big:
            # the producing unit's BN apply + residual + ReLU inside this conv's operand tile
            psc, psh, pres, pres_bn, side, side_mask = pro
            if pres_bn is None and psh.data_ptr() == psc.data_ptr() + 4 * psc.numel():  # BNState rows scale, shift
                coef = torch.as_strided(psc, (2, psc.numel()), (psc.numel(), 1))
            else:
                # [scale | shift (| residual scale | residual shift)] by device copies (no torch kernel)
                parts = [psc, psh] + ([pres_bn[0], pres_bn[1]] if pres_bn is not None else [])
                coef = K.concat_(torch.empty(sum(t.numel() for t in parts), dtype=torch.float32, device=psc.device),
                                 [t.contiguous() for t in parts])
            w4 = P.c[c.name + "_conv/kernel"]
            y, partial, T = G.conv_fwd_bnpro(x, w4, coef, pres, side, side_mask, proj=pres_bn is not None)
            x = side  # the unit's input as the backward needs it
        elif pro is not None or (not use8 and self._pw_part("plain") and self._pw_fwd_ok(c, False)):
            w2 = P.c[c.name + "_conv/kernel"].view(c.cout, c.cin_store)
            if pro is not None:
                psc, psh, pres, pres_bn, side, side_mask = pro
                rs, rb = pres_bn if pres_bn is not None else (None, None)
                y, partial, T = G.pw_conv(x, w2, prologue=("bn_fwd", psc, psh, pres, rs, rb, side, side_mask),
                                          stat=True)
                x = side  # the unit's input as the backward needs it
            else:
                y, partial, T = G.pw_conv(x, w2, stat=True)
        elif use8:
            xq, xslot = x8
            self._x8[c.name] = x8  # the fp8 weight gradient reuses the quantised input
            ws = self._w8_slots[self._w8_slot[c.name]]
            if G.conv_fwd4k8_pays(tuple(xq.shape), tuple(self._w8[c.name].shape), (c.stride, c.stride), (c.pad, c.pad)):
                # the 4-wave fp8 kernel on the long-reduction shapes (BN statistics per 128 rows)
                y, partial, T = G.conv_fwd4k8(xq, self._w8[c.name], (c.stride, c.stride), (c.pad, c.pad),
                                              ascale=(xslot[3:4], ws[3:4]))
            else:
                partial = torch.empty((T, 2, c.cout), dtype=torch.float32, device=x.device)
                y = G.conv_fwd_fp8(xq, self._w8[c.name], (c.stride, c.stride), (c.pad, c.pad), stat=partial,
                                   ascale=(xslot[3:4], ws[3:4]))
        elif bm == 256 and G.conv_fwd4w_pays(tuple(x.shape), tuple(P.var[c.name + "_conv/kernel"].shape),
                                             (c.stride, c.stride), (c.pad, c.pad)):
            # the 4-wave GEMM (SCHED 3 loop, im2col gather by the operand DMA, BN statistics from
            # its register epilogue per 128 rows): tools/conv1x1_g4_bench.py, BASELINE round 6
            y, partial, T = G.conv_fwd4w(x, P.c[c.name + "_conv/kernel"], (c.stride, c.stride), (c.pad, c.pad))
        else:
            partial = torch.empty((T, 2, c.cout), dtype=torch.float32, device=x.device)
            y = G.conv_fwd(x, P.c[c.name + "_conv/kernel"], (c.stride, c.stride), (c.pad, c.pad), stat=partial,
                           tile=(bm, bn))
        st = K.BNState(c.cout, x.device)
        pre = c.name + "_bn/"
        K.bn_fwd_stats(partial, T, M, P.var[pre + "gamma"], P.var[pre + "beta"], self.bn_eps, self.bn_momentum,
                       P.var[pre + "moving_mean"], P.var[pre + "moving_variance"], st)
        if pool:
            pooled, arg, mask = K.bn_relu_maxpool(y, st.scale, st.shift)
            return pooled, (x, y, mask, st), arg
        if defer:
            return y, [x, y, None, st]
        y2 = y.view(M, c.cout)
        mask = torch.empty(M * c.cout // 8, dtype=torch.uint8, device=x.device) if relu else None
        q8 = slot = None
        if want8:
            q8 = torch.empty((N, Pp, Q, c.cout), dtype=torch.uint8, device=x.device)
            slot = self._new_a_slot()
        out = K.bn_apply(y2, st.scale, st.shift, residual=None if residual is None else residual.view(M, c.cout),
                         residual_bn=residual_bn, relu=relu, mask=mask, q8=q8, q8_slot=slot,
                         store_out=store_out or not want8)
        if out is None:
            # only the fp8 copy exists: a storage-free stand-in that carries the shape (its consumer
            # reads x8; _wgrad refuses a bf16 weight gradient over it)
            out = torch.empty((1,), dtype=torch.bfloat16, device=x.device).expand(N, Pp, Q, c.cout)
        else:
            out = out.view(N, Pp, Q, c.cout)
        if want8:
            return out, [x, y, mask, st], (q8, slot)
        return out, [x, y, mask, st]

    def _convbn_bwd(self, c: ConvSpec, dout, ctx, need_dx=True, g_out=None, dx=None, dx_beta=0, dstat=None,
                    feeds=None, feeds2=None, sampled_only=False, dx_sampled=False, wgrad_last=False):
        """Backward of one conv+BN(+ReLU) unit. dout: gradient of the unit's output; with
        dstat = (partial, T) it is already ReLU-masked and its BN-backward sums came from the
        producing dgrad's epilogue. feeds: ctx of the conv+BN unit whose output is this conv's
        input — the dgrad epilogue then emits that unit's masked gradient + sums; feeds2: a
        second unit (projection shortcut BN) fed by the same gradient, whose sums come back as
        the third element of dstat_of_dx. sampled_only: a strided 1x1 dgrad leaves the pixels
        it does not sample unwritten (no zero fill); dx_sampled: dx (accumulated with dx_beta)
        is such a gradient, read only at its sampled (even h, w) pixels.
        Returns (dx, dstat_of_dx)."""
        from ..ops import gemm as G
        from ..ops import kernels as K
        P = self.params
        x, y, mask, st = ctx
        N, Pp, Q, Kc = y.shape
        M = N * Pp * Q
        pre = c.name + "_bn/"
        wname = c.name + "_conv/kernel"
        wshape = tuple(P.var[wname].shape)
        stem_k = (self.stem_kernel and c is self.stem
                  and G.stem_wgrad_ok(tuple(x.shape), wshape, (c.stride, c.stride), (c.pad, c.pad), self.in_channels))
        if (not need_dx and dstat is not None and self.fuse_bn_bwd
                and (stem_k or G.conv_wgrad_bn_fusable(tuple(x.shape), wshape, (c.stride, c.stride), (c.pad, c.pad)))):
            # weight gradient only (the stem): the BN backward is applied inside the weight
            # gradient's operand load, its output never stored (one HBM pass less at the very end
            # of the backward, where nothing else runs)
            coef = K.bn_backward_coef(M, Kc, P.var[pre + "gamma"], st, P.g[pre + "gamma"], P.g[pre + "beta"],
                                      dstat[0], dstat[1])
            if stem_k:
                G.stem_wgrad(x, dout, y, coef, out=P.g[wname])  # dedicated kernel (stem_wgrad.hip)
            else:
                G.conv_wgrad_bn(x, dout, y, coef, wshape, (c.stride, c.stride), (c.pad, c.pad), out=P.g[wname])
            if self._wgrad_stream is not None:
                # the bucket this completes may hold side-stream gradients: collectives issued
                # from here must order after that stream too
                graphs.join(torch.cuda.current_stream(), self._wgrad_stream)
            self._ready(c.name + "_bn/moving_variance")
            return None, None
        if (need_dx and wgrad_last and dstat is not None and feeds is None and dx is None and not sampled_only
                and self.fuse_bn_bwd and self.pw_wgrad and self._pw_part("dgrad") and self._pw_dgrad_ok(c)
                and G.pw_wgrad_fusable(M, c.cin_store, Kc, False)):
            # the unit-stride projection shortcut (stage 2): BN backward, data and weight gradient
            # in one streaming kernel (no dz pass, no dz store, no weight-gradient re-read)
            coef = K.bn_backward_coef(M, Kc, P.var[pre + "gamma"], st, P.g[pre + "gamma"], P.g[pre + "beta"],
                                      dstat[0], dstat[1])
            wt2 = self._crsk(wname).view(c.cin_store, c.cout)
            out = G.pw_conv(dout, wt2, prologue=("bn_bwd", y, None, coef, None),
                            wgrad=(x, P.g[wname].view(c.cout, c.cin_store)), max_wgs=self.side_pw_wgs)
            self._cd_done = graphs.mark(torch.cuda.current_stream())
            return out, None
        if (need_dx and dstat is not None and feeds is None and not wgrad_last and not sampled_only and not dx_sampled
                and self.fuse_bn_bwd and self.pw_wgrad and self._pw_part("dgrad") and self.device.type == "cuda"
                and c.k == 1 and c.stride == 1 and c.pad == 0
                and G.pw_wgrad_fusable(M, c.cin_store, Kc, bool(dx is not None and dx_beta))):
            # a 1x1 unit whose input is not a BN unit's output (stage 2's first c1, fed by the max
            # pool; accumulating into the projection's gradient): BN backward, data and weight
            # gradient in one streaming kernel
            coef = K.bn_backward_coef(M, Kc, P.var[pre + "gamma"], st, P.g[pre + "gamma"], P.g[pre + "beta"],
                                      dstat[0], dstat[1])
            wt2 = self._crsk(wname).view(c.cin_store, c.cout)
            out = G.pw_conv(dout, wt2, prologue=("bn_bwd", y, None, coef, None), out=dx,
                            beta=dx_beta if dx is not None else 0, wgrad=(x, P.g[wname].view(c.cout, c.cin_store)),
                            fold_stream=self._fold_stream(), keep=self._side_keep)
            self._ready_main(c.name + "_bn/moving_variance")
            return out, None
        g8_take = self._g8_take(c, need_dx, feeds, feeds2, dx, dx_beta, dx_sampled)
        if (need_dx and dstat is not None and feeds is not None and feeds2 is None and not g8_take
                and self.fuse_bn_bwd and self._pw_part("dgrad") and self._pw_dgrad_ok(c)):
            # BN backward applied inside the data gradient's operand load (streaming pointwise
            # kernel): dz is written once there for the weight gradient, never re-read by the dgrad
            coef = K.bn_backward_coef(M, Kc, P.var[pre + "gamma"], st, P.g[pre + "gamma"], P.g[pre + "beta"],
                                      dstat[0], dstat[1])
            wt2 = self._crsk(wname).view(c.cin_store, c.cout)
            _, fy, fmask, _ = feeds
            bs2 = (x.shape[1], x.shape[2]) if dx_sampled else None
            if self.pw_wgrad and G.pw_wgrad_fusable(M, c.cin_store, Kc):
                # ... and the weight gradient in the same kernel, from the dz tile in LDS: dz is
                # never stored, the side-stream pass re-reading dz and x disappears
                out, partial, T = G.pw_conv(dout, wt2, prologue=("bn_bwd", y, None, coef, None), bn_stat=(fy, fmask),
                                            out=dx, beta=dx_beta if dx is not None else 0, beta_s2=bs2,
                                            wgrad=(x, P.g[wname].view(c.cout, c.cin_store)),
                                            fold_stream=self._fold_stream(), keep=self._side_keep)
                self._ready_main(c.name + "_bn/moving_variance")
                return out, (partial, T)
            dz = torch.empty_like(y)
            out, partial, T = G.pw_conv(dout, wt2, prologue=("bn_bwd", y, None, coef, dz), bn_stat=(fy, fmask),
                                        out=dx, beta=dx_beta if dx is not None else 0, beta_s2=bs2)
            self._wgrad(c, x, dz, wname)
            return out, (partial, T)
        unstored = c.name in self._x_unstored  # only the fp8 copy of x exists: the fp8 branch below
        if (need_dx and dstat is not None and feeds is not None and feeds2 is None and dx is None and not unstored
                and self.fuse_bn_bwd and self.c3_dgrad == 1 and self._c3_ok(c, x.shape[1], x.shape[2])):
            # halo 3x3 data gradient with this unit's BN backward as its operand prologue (dz is
            # written once there for the weight gradient) and the feeding unit's BN-backward
            # statistics in its epilogue
            coef = K.bn_backward_coef(M, Kc, P.var[pre + "gamma"], st, P.g[pre + "gamma"], P.g[pre + "beta"],
                                      dstat[0], dstat[1])
            dz = torch.empty_like(y)
            wt = self._crsk(wname)
            _, fy, fmask, _ = feeds
            out, partial, T = G.conv3_halo(dout, wt, flip=True, prologue=("bn_bwd", y, None, coef, dz),
                                           bn_stat=(fy, fmask))
            self._wgrad(c, x, dz, wname)
            return out, (partial, T)
        stride, pad = (c.stride, c.stride), (c.pad, c.pad)
        if (need_dx and dstat is not None and self.fuse_bn_bwd and self.bn_pro and not wgrad_last and not sampled_only
                and not unstored and not g8_take
                and self.device.type == "cuda" and Kc <= self.BNPRO_MAX_K and c.cin_store <= self.BNPRO_MAX_N
                and G.dgrad_bnpro_ok(tuple(x.shape), (c.cin_store, c.k, c.k, Kc), stride, pad)):
            # BN backward formed inside the data gradient's operand tile (dz stored there once for
            # the weight gradient, which therefore starts after this launch)
            coef = K.bn_backward_coef(M, Kc, P.var[pre + "gamma"], st, P.g[pre + "gamma"], P.g[pre + "beta"],
                                      dstat[0], dstat[1])
            dz = torch.empty_like(y)
            wt = self._crsk(wname)
            bs2 = (x.shape[1], x.shape[2]) if dx_sampled else None
            pro = (y, coef, dz)
            if feeds is not None and G.dgrad_stat_rows(tuple(x.shape), tuple(wt.shape), stride, pad) is not None:
                _, fy, fmask, _ = feeds
                if feeds2 is not None:
                    out, partial, T, partial2 = G.conv_dgrad(dout, wt, x.shape, stride, pad, out=dx, beta=dx_beta,
                                                             bn_stat=(fy, fmask), bn_stat2=feeds2[1], beta_s2=bs2,
                                                             bn_pro=pro)
                    self._wgrad(c, x, dz, wname)
                    return out, (partial, T, partial2)
                out, partial, T = G.conv_dgrad(dout, wt, x.shape, stride, pad, out=dx, beta=dx_beta,
                                               bn_stat=(fy, fmask), beta_s2=bs2, bn_pro=pro)
                self._wgrad(c, x, dz, wname)
                return out, (partial, T)
            out = G.conv_dgrad(dout, wt, x.shape, stride, pad, out=dx, beta=dx_beta, beta_s2=bs2, bn_pro=pro)
            self._wgrad(c, x, dz, wname)
            return out, None
        dz8 = None
        wgrad_done = False
        if dstat is not None:
            # (dx given: a c1 data gradient accumulating into the shortcut gradient, beta = 1)
            g8 = g8_take
            # fp8 weight gradient without an fp8 data gradient (strided 3x3): dz8 still produced
            # from the first step on (the slot collects its amax), consumed from the second
            # Also whenever the forward stored only the fp8 copy of x (_x8_only) but the fp8 data
            # gradient is off for this conv this step (e.g. TTD_WPREP=0: no prepared e4m3 filters):
            # the bf16 weight gradient has no input to read, so dz8 is produced for the fp8 one.
            gw8 = (not g8 and self._fp8 is not None and c.name in self._gq
                   and (c.name not in self._g8 or c.name in self._x_unstored)
                   and not wgrad_last and self._fp8_wgrad_ok(c, tuple(x.shape)))
            q8 = torch.empty(y.numel(), dtype=torch.uint8, device=y.device) if (g8 or gw8) else None
            gslot = self._g_slots[self._gq[c.name]] if q8 is not None else None
            # both consumers of dz on fp8 (data gradient and weight gradient): no bf16 dz at all
            w8 = g8 and self._fp8_bwd_steps >= 1 and not wgrad_last and self._fp8_wgrad_ok(c, tuple(x.shape))
            dz = K.bn_backward_from_partial(dout.view(M, Kc), y.view(M, Kc), P.var[pre + "gamma"], st,
                                            P.g[pre + "gamma"], P.g[pre + "beta"], dstat[0], dstat[1], q8=q8,
                                            q8_slot=gslot, store_dz=not w8)
            if dz is not None:
                dz = dz.view(N, Pp, Q, Kc)
            if g8 and self._fp8_bwd_steps >= 1:  # (step 0 only collects the gradient amax)
                dz8 = q8.view(N, Pp, Q, Kc)
                if w8:
                    self._wgrad(c, x, dz, wname, fp8=(self._x8[c.name], dz8, gslot))
                    wgrad_done = True
            elif gw8 and self._fp8_bwd_steps >= 1:
                self._wgrad(c, x, dz, wname, fp8=(self._x8[c.name], q8.view(N, Pp, Q, Kc), gslot))
                wgrad_done = True
        else:
            dz = K.bn_backward(dout.view(M, Kc), None, y.view(M, Kc), P.var[pre + "gamma"], st, P.g[pre + "gamma"],
                               P.g[pre + "beta"], g_out=None if g_out is None else g_out.view(M, Kc),
                               mask=mask).view(N, Pp, Q, Kc)
        if not wgrad_last and not wgrad_done:
            self._wgrad(c, x, dz, wname)
        if not need_dx:
            return None, None
        wt = self._crsk(wname)
        bs2 = (x.shape[1], x.shape[2]) if dx_sampled else None
        if dz8 is not None:
            # fp8 data gradient (e5m2 dz x e4m3 transposed filter) with the feeding unit's masked
            # gradient + BN-backward sums in its epilogue
            _, fy, fmask, _ = feeds
            kind, off, shape = self._wp_cur._views[wname]
            wt8 = self._wt8_buf[off:off + int(np.prod(shape))].view(shape)
            i8 = self._g8[c.name]
            out, partial, T = G.conv_dgrad_fp8(dz8, wt8, x.shape, stride, pad, bn_stat=(fy, fmask),
                                               ascale=(self._g_slots[i8][3:4], self._wt8_slots[i8][3:4]),
                                               out=dx, beta=dx_beta if dx is not None else 0, beta_s2=bs2)
            return out, (partial, T)
        if (feeds is not None and feeds2 is None and dx is None and self.fuse_bn_bwd and self.c3_dgrad == 2
                and self._c3_ok(c, x.shape[1], x.shape[2])):
            # halo 3x3 kernel (flipped filter) with the feeding unit's BN-backward sums in its epilogue
            _, fy, fmask, _ = feeds
            out, partial, T = G.conv3_halo(dz, wt, flip=True, bn_stat=(fy, fmask))
            return out, (partial, T)
        if (feeds is not None and self.fuse_bn_bwd
                and G.dgrad_stat_rows(tuple(x.shape), tuple(wt.shape), stride, pad) is not None):
            _, fy, fmask, _ = feeds
            if feeds2 is not None and stride == (1, 1):
                out, partial, T, partial2 = G.conv_dgrad(dz, wt, x.shape, stride, pad, out=dx, beta=dx_beta,
                                                         bn_stat=(fy, fmask), bn_stat2=feeds2[1], beta_s2=bs2)
                return out, (partial, T, partial2)
            out, partial, T = G.conv_dgrad(dz, wt, x.shape, stride, pad, out=dx, beta=dx_beta, bn_stat=(fy, fmask),
                                           beta_s2=bs2, ws=self._phase_ws(wname))
            return out, (partial, T)
        out = G.conv_dgrad(dz, wt, x.shape, stride, pad, out=dx, beta=dx_beta, sampled_only=sampled_only, beta_s2=bs2,
                           ws=self._phase_ws(wname))
        if wgrad_last:
            # data gradient first (its consumer waits on this event), then the weight gradient
            self._cd_done = graphs.mark(torch.cuda.current_stream())
            # its gradient-ready hook waits for the caller: the variables before it in the flat
            # layout (the block's c3 and c2) are not final yet
            self._wgrad(c, x, dz, wname, ready=False)
        return out, None

    def _weight_prep(self, image_shape):
        """Data-gradient filter operands of every conv, prepared in one launch at the start of the
        step (ops.kernels.WeightPrep): [C,R,S,K] transposes, plus the sub-pixel phase filters of
        the strided 3x3 convs (their geometry depends on the image size). TTD_WPREP=0: per-conv
        transposes / phase gathers inside the backward, as before."""
        from ..ops import kernels as K
        key = tuple(image_shape[1:3])
        if getattr(self, "_wp_key", None) == key:
            return self._wp
        P = self.params
        wp = K.WeightPrep(P.compute)
        H = (image_shape[1] + 2 * self.stem.pad - self.stem.k) // self.stem.stride + 1
        W = (image_shape[2] + 2 * self.stem.pad - self.stem.k) // self.stem.stride + 1
        H, W = K.pool_out(H, 3, 2, 1), K.pool_out(W, 3, 2, 1)
        for blk in self.blocks:
            for key_ in ("c1", "c2", "c3", "cd"):
                c = blk[key_]
                if c is None:
                    continue
                name = c.name + "_conv/kernel"
                shape = tuple(P.var[name].shape)
                wp.add(name, P.offsets[name], shape)
                if c.k > 1 and c.stride > 1:
                    wp.add(name + "/phases", P.offsets[name], shape, sub=(c.stride, c.pad, c.pad, H, W))
            s = blk["c2"].stride
            H, W = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
        self._wp = wp.build()
        self._wp_key = key
        if self._fp8 is not None and self._g8:
            # e4m3 copies of the fp8-dgrad convs' transposed filters, quantised from the WeightPrep
            # buffer (same element offsets) with current per-tensor scaling
            rows = []
            for c in self.conv_list():
                if c.name in self._g8:
                    kind, off, shape = wp._views[c.name + "_conv/kernel"]
                    rows.append((off, int(np.prod(shape)), self._g8[c.name]))
            arr = np.zeros(len(rows), dtype=np.dtype([("off", "<i8"), ("len", "<i4"), ("slot", "<i4")]))
            for i, r in enumerate(rows):
                arr[i] = r
            self._wt8_table = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)
            self._wt8_n, self._wt8_max = len(rows), max(r[1] for r in rows)
            self._wt8_buf = torch.empty(wp.buf.numel(), dtype=torch.uint8, device=self.device)
            self._wt8_slots = torch.zeros((len(self._g8), K.FP8_SLOT), dtype=torch.float32, device=self.device)
        return self._wp

    def _crsk(self, wname):
        from ..ops import kernels as K
        wp = self._wp_cur
        if wp is not None and wp.has(wname):
            return wp.crsk(wname)
        return K.krsc_to_crsk(self.params.c[wname])

    def _phase_ws(self, wname):
        wp = self._wp_cur
        if wp is not None and wp.has(wname + "/phases"):
            return wp.phases(wname + "/phases")
        return None

    def _x8_only(self, c: ConvSpec, x_shape) -> bool:
        """The forward may skip the bf16 copy of c's input: c runs its forward on the fp8 copy and
        this step's backward will take its weight gradient from it too (a fp8 dz exists from the
        second step on). TTD_FP8_ONLY_INPUT=0 keeps the bf16 copy."""
        from ..ops import gemm as G
        return (self.fp8_only_input and self.fp8_wgrad and self._fp8 is not None and self._fp8_bwd_steps >= 1
                and self._fp8_conv(c) and c.name in self._gq and (c.k > 1 or self.fp8_1x1_wgrad)
                and G.conv_wgrad_fp8_ok(tuple(x_shape), tuple(self.params.var[c.name + "_conv/kernel"].shape),
                                        (c.stride, c.stride), (c.pad, c.pad)))

    def _fp8_wgrad_ok(self, c: ConvSpec, x_shape) -> bool:
        """c's weight gradient runs on fp8 (ops.gemm.conv_wgrad_fp8) in this step's backward: the
        fp8 forward quantised its input and the fp8 data gradient quantises its dz."""
        from ..ops import gemm as G
        return (self.fp8_wgrad and self._fp8 is not None and c.name in self._gq and c.name in self._x8
                and (c.k > 1 or self.fp8_1x1_wgrad)
                and G.conv_wgrad_fp8_ok(tuple(x_shape), tuple(self.params.var[c.name + "_conv/kernel"].shape),
                                        (c.stride, c.stride), (c.pad, c.pad)))

    def _wgrad(self, c: ConvSpec, x, dz, wname, ready=True, fp8=None):
        """Weight gradient of conv c into its flat gradient slice; on the side stream when enabled,
        concurrent with the data-gradient chain (fills the tail waves of the 1-workgroup-per-CU
        GEMMs), then the gradient-ready hook (collectives order after the side stream).
        fp8 = (x8, dz8, dz8's scale slot): the fp8 weight gradient from the quantised copies (x8 =
        (codes, slot) of the fp8 forward) instead of the bf16 x and dz."""
        from ..ops import gemm as G
        P = self.params
        side = self._wgrad_stream

        def run():
            if fp8 is not None:
                (xq, xslot), dz8, gslot = fp8
                G.conv_wgrad_fp8(xq, dz8, tuple(P.var[wname].shape), (c.stride, c.stride), (c.pad, c.pad),
                                 ascale=(gslot[3:4], xslot[3:4]), out=P.g[wname])
            else:
                if c.name in self._x_unstored:
                    raise RuntimeError("%s: bf16 weight gradient asked for, but the forward stored only the fp8 "
                                       "copy of its input" % c.name)
                G.conv_wgrad(x, dz, tuple(P.var[wname].shape), (c.stride, c.stride), (c.pad, c.pad), out=P.g[wname])
            if ready:
                self._ready(c.name + "_bn/moving_variance")  # last variable of this conv's group

        if side is not None:
            if torch.cuda.current_stream() != side:  # (a stream waiting on its own event breaks hipGraph capture)
                graphs.fork(torch.cuda.current_stream(), side)
            with torch.cuda.stream(side):
                run()
            # keep the operands alive until the streams join at the end of the backward (no
            # record_stream: its deferred frees made the allocator re-malloc when the host ran
            # several steps ahead)
            self._side_keep += [t for t in (x, dz) if t is not None] + ([fp8[0][0], fp8[1]] if fp8 is not None else [])
        else:
            run()

    def _fold_stream(self):
        """Stream for the slab fold of a main-stream fused weight gradient (pw_conv wgrad=): the
        side stream, unless disabled (TTD_PW_FOLD_SIDE=0) or already the current stream. On the
        main stream the fold waited ~1 ms per launch for CUs held by the side stream's weight
        gradients (profiles/r4_resnet50_b1024_step_streams_graph.txt)."""
        side = self._wgrad_stream
        if side is None or not self.pw_fold_side or torch.cuda.current_stream() == side:
            return None
        return side

    def _ready(self, name):
        if self._grad_hook is not None:
            self._grad_hook(name)

    def _ready_main(self, name):
        """Gradient-ready hook for a gradient produced on the main stream: issued from the side
        stream after a fork, so the bucket it completes also orders after the side-stream
        weight gradients queued before it (flat-layout order)."""
        side = self._wgrad_stream
        if self._grad_hook is None:
            return
        if side is None:
            self._grad_hook(name)
            return
        graphs.fork(torch.cuda.current_stream(), side)
        with torch.cuda.stream(side):
            self._grad_hook(name)

    def forward_backward(self, images, labels, grad_scale: Optional[float] = None, grad_hook=None):
        """One training forward + backward on the GPU engine.

        images: [N, H, W, in_channels] bf16 (NHWC); labels: [N] int. Writes every trainable
        gradient into params.grad; returns a device fp32[2] = (mean loss, mean accuracy).
        grad_hook(name) is called as soon as the gradients of every variable up to and
        including `name` (in flat-layout order) are final — the bucketed all-reduce cut points.
        """
        from ..ops import gemm as G
        from ..ops import kernels as K
        self._grad_hook = grad_hook
        P = self.params
        N = images.shape[0]
        self._wgrad_stream = None
        self._side_keep = []
        if self.wgrad_stream:
            if getattr(self, "_side", None) is None:
                side_cus = int(os.environ.get("TTD_SIDE_CUS", "0"))
                # TTD_SIDE_CUS > 0: the side stream may only occupy that many CUs (utils.graphs)
                self._side = (graphs.cu_masked_stream(self.device, side_cus) if side_cus > 0
                              else torch.cuda.Stream(device=self.device))
            self._wgrad_stream = self._side
        if grad_scale is None:
            grad_scale = 1.0 / N
        fp8 = self._fp8 is not None
        if images.shape[-1] == self.in_store or self._stem_packed_ok(tuple(images.shape)):
            x = images  # the dedicated stem kernels read the packed RGB (no channel-padding pass)
        else:
            x = K.pad_channels(images.contiguous(), self.in_store)
        self._x8 = {}
        self._x_unstored = set()
        if fp8:
            self._fp8_step_begin()
        self._wp_cur = None
        if self.wprep and self.device.type == "cuda":
            # this step's data-gradient filters (the weights are final until the optimizer runs)
            self._wp_cur = self._weight_prep(tuple(images.shape))
            self._wp_cur.run()
            if fp8 and self._g8:
                K.fp8_quant_weights(self._wp_cur.buf, self._wt8_buf, self._wt8_table, self._wt8_n, self._wt8_max,
                                    self._wt8_slots)

        def unit(c, inp, relu, residual=None, inp8=None, want8=False, defer=False, residual_bn=None, pro=None,
                 pro_big=False, consumer=None):
            # consumer: the conv this unit's output feeds; when that conv will take both its forward
            # and its weight gradient from the fp8 copy, the bf16 output is never stored
            only8 = False
            if want8 and consumer is not None:
                n_, h_, w_ = inp.shape[:3]
                oshape = (n_, (h_ + 2 * c.pad - c.k) // c.stride + 1, (w_ + 2 * c.pad - c.k) // c.stride + 1, c.cout)
                only8 = self._x8_only(consumer, oshape)
            r = self._convbn_fwd(c, inp, relu, residual=residual, x8=inp8, want8=want8, defer=defer,
                                 residual_bn=residual_bn, pro=pro, pro_big=pro_big, store_out=not only8)
            if only8:
                self._x_unstored.add(consumer.name)
            return r if want8 else (r[0], r[1], None)

        from ..utils import tracing
        fwd_range = tracing.range("resnet/forward")
        fwd_range.__enter__()
        # ---- forward
        stem_shape = (N, (x.shape[1] + 2 * self.stem.pad - self.stem.k) // self.stem.stride + 1,
                      (x.shape[2] + 2 * self.stem.pad - self.stem.k) // self.stem.stride + 1, self.stem.cout)
        pool_fused = self.fuse_bn_bwd and K.stem_pool_fusable(stem_shape)
        if pool_fused:
            h, s_ctx, arg = self._convbn_fwd(self.stem, x, relu=True, pool=True)
        else:
            s_out, s_ctx = self._convbn_fwd(self.stem, x, relu=True)
            h, arg = K.maxpool_fwd(s_out, 3, 2, 1)
        h8 = None
        ctxs = []
        # pend: the previous block's c3 unit whose BN apply (+ residual, ReLU) is deferred into this
        # block's c1 conv (streaming pointwise kernel prologue): (y3, state, residual, residual_bn, ctx)
        pend = None
        for i, blk in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            side = self._wgrad_stream
            c1 = None
            # c2 on the halo kernel: c1's BN apply + ReLU run inside c2's operand load
            c3ok = not self._fp8_conv(blk["c2"]) and self._c3_ok(blk["c2"], h.shape[1] if pend is None else pend[0].shape[1],
                                                                 h.shape[2] if pend is None else pend[0].shape[2])
            if pend is not None:
                # this block's input h = relu(bn3(y3) + shortcut) is produced by c1's operand load
                y3p, stp, resp, resbnp, ctxp, pbig = pend
                h = torch.empty_like(y3p)
                hm = torch.empty(h.numel() // 8, dtype=torch.uint8, device=h.device)
                ctxp[2] = hm  # the producing unit's ReLU bits (its backward reads them)
                o1, c1, o1_8 = unit(blk["c1"], y3p, True, pro=(stp.scale, stp.shift, resp, resbnp, h, hm), defer=c3ok,
                                    want8=fp8 and not c3ok and self._fp8_conv(blk["c2"]), pro_big=pbig,
                                    consumer=blk["c2"])
                pend = None
            proj_side = blk["cd"] is not None and side is not None and self.fwd_proj_side
            if proj_side:
                # projection shortcut on the side stream, concurrent with the c1 -> c2 chain
                main = torch.cuda.current_stream()
                graphs.fork(main, side)
                with torch.cuda.stream(side):
                    sc, cd, _ = unit(blk["cd"], h, False, inp8=h8, defer=self.fuse_proj)
                # h / h8 stay referenced (c1's ctx) past the join below; cd's outputs were made on
                # the side stream, whose next work is always ordered after this step's main stream
            if c1 is None:
                o1, c1, o1_8 = unit(blk["c1"], h, True, inp8=h8, want8=fp8 and self._fp8_conv(blk["c2"]), defer=c3ok,
                                    consumer=blk["c2"])
            pro2 = None
            if c3ok:
                # o1 was returned raw (deferred BN): the halo kernel writes the applied o1 + bits
                y1 = o1
                o1 = torch.empty_like(y1)
                c1[2] = torch.empty(o1.numel() // 8, dtype=torch.uint8, device=o1.device)
                pro2 = (c1[3].scale, c1[3].shift, None, None, o1, c1[2])
                o1 = y1  # c2's operand is the raw c1 output; _convbn_fwd swaps in the applied one
            fuse23 = self._pw_part("c23") and self._pw_fwd_ok(blk["c3"], True)
            if fuse23:
                # c2's BN + ReLU are applied inside c3's operand load; o2 and its ReLU bits are
                # written there (c3's weight gradient and c2's backward read them)
                y2, c2, _ = unit(blk["c2"], o1, True, inp8=o1_8, defer=True, pro=pro2)
                o2 = torch.empty_like(y2)
                c2[2] = torch.empty(o2.numel() // 8, dtype=torch.uint8, device=o2.device)
                o2_8 = None
            else:
                # (the last block's c3 gets its output gradient from the pooling backward without
                # BN sums: that path has no e5m2 dz, so its bf16 input stays stored)
                o2, c2, o2_8 = unit(blk["c2"], o1, True, inp8=o1_8, want8=fp8 and self._fp8_conv(blk["c3"]), pro=pro2,
                                    consumer=blk["c3"] if nxt is not None else None)
            defer3 = (nxt is not None and self._pw_part("c31") and self._pw_fwd_ok(nxt["c1"], True)
                      and not self._fp8_conv(nxt["c1"]))
            c3_in = y2 if fuse23 else o2
            defer_big = False
            if not defer3 and nxt is not None:
                # or on the 256-row kernel's operand prologue (stage-3/4 widths)
                defer3 = defer_big = self._fwd_pro_ok(nxt["c1"], tuple(c3_in.shape[:3]) + (blk["c3"].cout,))
            # the shortcut is first read by c3's apply pass, or — when c3's BN apply is deferred into
            # the next block's c1 — only there: the join then waits until after c3 (the side-stream
            # projection gets c3's duration too; it measured 0.2-0.3 ms exposed before c3)
            late_join = proj_side and defer3 and self.late_proj_join
            if proj_side and not late_join:
                graphs.join(main, side)
            elif blk["cd"] is not None and not proj_side:
                sc, cd, _ = unit(blk["cd"], h, False, inp8=h8, defer=self.fuse_proj)
            elif blk["cd"] is None:
                sc, cd = h, None
            sc_bn = (cd[3].scale, cd[3].shift) if cd is not None and self.fuse_proj else None
            c3_pro = (c2[3].scale, c2[3].shift, None, None, o2, c2[2]) if fuse23 else None
            if defer3:
                y3, c3, _ = unit(blk["c3"], c3_in, True, defer=True, pro=c3_pro)
                if late_join:
                    graphs.join(main, side)
                pend = (y3, c3[3], sc, sc_bn, c3, defer_big)
                o3, h8 = None, None
            else:
                o3, c3, h8 = unit(blk["c3"], c3_in, True, residual=sc, inp8=o2_8, residual_bn=sc_bn, pro=c3_pro,
                                  want8=fp8 and nxt is not None and self._fp8_conv(nxt["c1"]))
            ctxs.append((c1, c2, c3, cd))
            h = o3
        feat_shape = h.shape
        pooled = K.avgpool_fwd(h)
        logits = G.gemm(pooled, P.c["predictions/kernel"], bias=P.var["predictions/bias"])
        sums, dlogits, _, _ = K.sparse_xent(logits, labels, grad_scale)
        fwd_range.__exit__(None, None, None)
        bwd_range = tracing.range("resnet/backward")
        bwd_range.__enter__()
        # ---- backward
        G.gemm(pooled, dlogits, trans_a=True, out=P.g["predictions/kernel"])
        K.colsum(dlogits, out=P.g["predictions/bias"])
        self._ready("predictions/bias")
        dpooled = G.gemm(dlogits, P.c["predictions/kernel"], trans_b=True)
        dh = K.avgpool_bwd(dpooled, feat_shape)
        dh_stat = None  # (partial, T) when dh is already the masked gradient of the block's c3 unit
        for i in reversed(range(len(self.blocks))):
            blk = self.blocks[i]
            c1, c2, c3, cd = ctxs[i]
            prev_c3 = ctxs[i - 1][2] if i > 0 else None  # the unit that produced this block's input
            prev_cd = ctxs[i - 1][3] if i > 0 else None  # its projection shortcut (fed by the same gradient)
            side = self._wgrad_stream
            cd_side = blk["cd"] is not None and dh_stat is not None and side is not None and self.cd_side
            sampled = False
            if blk["cd"] is not None:
                cd_stat = (dh_stat[2], dh_stat[1]) if dh_stat is not None and len(dh_stat) == 3 else None
                # a stride-2 projection writes only the pixels it samples; c1's accumulate reads it there
                sampled = self.sampled_dgrad and blk["cd"].stride != 1 and blk["cd"].pad == 0
            cd_done = None
            if cd_side:
                # projection branch (BN backward + strided dgrad, then its weight gradient) on the side
                # stream, concurrent with the c3 -> c2 chain; c1's dgrad below accumulates into dx
                graphs.fork(torch.cuda.current_stream(), side)
                self._cd_done = None
                with torch.cuda.stream(side):
                    dx, _ = self._convbn_bwd(blk["cd"], dh, cd, dstat=cd_stat, sampled_only=sampled, wgrad_last=True)
                    cd_done = self._cd_done
                assert cd_done is not None, "projection backward took a path without the wgrad_last event"
                # dx was made on the side stream and dh is read there: both alive until the streams join
                self._side_keep += [dx, dh]
            if dh_stat is not None:
                g_sc = dh  # already ReLU-masked by the producing dgrad epilogue
                d2, st2 = self._convbn_bwd(blk["c3"], dh, c3, dstat=dh_stat[:2], feeds=c2)
            else:
                g_sc = torch.empty_like(dh)
                d2, st2 = self._convbn_bwd(blk["c3"], dh, c3, g_out=g_sc, feeds=c2)
            d1, st1 = self._convbn_bwd(blk["c2"], d2, c2, dstat=st2, feeds=c1)
            if cd_done is not None:
                # c3 / c2 weight gradients are now queued on the side stream behind the projection's:
                # the bucket hook for the projection variables can fire (in flat-layout order)
                with torch.cuda.stream(side):
                    self._ready(blk["cd"].name + "_bn/moving_variance")
                graphs.join_mark(torch.cuda.current_stream(), cd_done)
            elif blk["cd"] is not None:
                dx, _ = self._convbn_bwd(blk["cd"], g_sc, cd, dstat=cd_stat, sampled_only=sampled)
            else:
                dx = g_sc
            dh, dh_stat = self._convbn_bwd(blk["c1"], d1, c1, dx=dx, dx_beta=1, dstat=st1, feeds=prev_c3,
                                           feeds2=prev_cd, dx_sampled=sampled)
        if pool_fused:
            g, partial, T = K.maxpool_bwd_bnstat(dh, arg, s_ctx[2], s_ctx[1])
            self._convbn_bwd(self.stem, g, s_ctx, need_dx=False, dstat=(partial, T))
        else:
            dstem = K.maxpool_bwd(dh, arg, s_out.shape, 3, 2, 1)
            self._convbn_bwd(self.stem, dstem, s_ctx, need_dx=False)
        if self._wgrad_stream is not None:
            graphs.join(torch.cuda.current_stream(), self._wgrad_stream)
            self._wgrad_stream = None
        self._side_keep = []
        if fp8:
            self._fp8_bwd_steps += 1
        bwd_range.__exit__(None, None, None)
        self._grad_hook = None
        return sums

    # ----------------------------------------------------------------- reference (CPU / oracle)
    def reference_loss(self, images, labels, params=None, bf16_activations=False):
        """fp32 PyTorch implementation of the same network (NCHW internally), used on CPU and
        as the numerics oracle for the GPU engine. Returns (loss, accuracy, logits); BN uses
        batch statistics (training mode) and does not touch the moving averages.

        bf16_activations=True rounds every tensor the GPU engine stores in bf16 (conv outputs,
        unit outputs, pooled features, logits) with a straight-through estimator, so the
        oracle follows the engine's rounding points and only accumulation order differs."""
        P = params if params is not None else {n: self.params.var[n] for n in self.params.names()}
        x = images.float().permute(0, 3, 1, 2)

        def rnd(t):
            if not bf16_activations:
                return t
            return t + (t.to(torch.bfloat16).float() - t).detach()

        def convbn(c, t, relu, res=None):
            w = P[c.name + "_conv/kernel"][..., :t.shape[1]].permute(0, 3, 1, 2)
            y = rnd(F.conv2d(t, w, stride=c.stride, padding=c.pad))
            y = F.batch_norm(y, None, None, P[c.name + "_bn/gamma"], P[c.name + "_bn/beta"], training=True,
                             eps=self.bn_eps)
            if res is not None:
                y = y + res
            return rnd(F.relu(y) if relu else y)

        h = convbn(self.stem, x, True)
        h = F.max_pool2d(h, 3, 2, 1)
        for blk in self.blocks:
            o = convbn(blk["c1"], h, True)
            o = convbn(blk["c2"], o, True)
            sc = convbn(blk["cd"], h, False) if blk["cd"] is not None else h
            h = convbn(blk["c3"], o, True, sc)
        pooled = rnd(h.mean((2, 3)))
        logits = rnd(pooled @ P["predictions/kernel"] + P["predictions/bias"])
        loss = F.cross_entropy(logits, labels.long())
        acc = (logits.argmax(1) == labels.long()).float().mean()
        return loss, acc, logits

    def reference_forward_backward(self, images, labels, grad_scale=None):
        """CPU training step: autograd through reference_loss, gradients written to the flat
        gradient buffer (same contract as forward_backward)."""
        P = self.params
        leaves = {n: P.var[n].detach().clone().requires_grad_(P.spec(n).trainable) for n in P.names()}
        loss, acc, _ = self.reference_loss(images, labels, leaves)
        scale = 1.0 if grad_scale is None else grad_scale * images.shape[0]
        (loss * scale).backward()
        with torch.no_grad():
            for n, t in leaves.items():
                if t.grad is not None:
                    P.g[n].copy_(t.grad)
        return torch.stack([loss.detach(), acc.detach()])


def resnet50(num_classes=1000, device="cuda", **kw) -> ResNet:
    """ResNet-50 v1.5; precision="fp8" for the fp8 forward path (config 5)."""
    return ResNet(STAGES_50, num_classes=num_classes, device=device, **kw)
