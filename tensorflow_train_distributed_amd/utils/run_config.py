"""Typed run configuration: one dataclass for what a training or benchmark run
needs beyond the model — batch, steps, precision, optimizer, LR schedule, data-parallel
communication, hipGraph, checkpoint / summary cadence — overridable from the command line,
from a JSON/YAML file and from `TTD_RUN_<FIELD>` environment variables.

The reference keeps these as module constants and five tf.app.flags
(/root/reference/distribute_training.py:10-36: batch_size 128, learning_rate 0.01, decay 0.96
every 500 steps, 10000 training steps, checkpoint every 60 s, summaries every 100 steps);
`RunConfig.reference_mnist()` reproduces them. tf.estimator.RunConfig's cadence fields keep
their TF names (save_checkpoints_secs, save_summary_steps, log_step_count_steps).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class RunConfig:
    model: str = "resnet50"            # resnet50 | bert | mlp
    per_replica_batch: int = 0         # 0 = the model's default (1024 images / 128 sequences / 128 examples)
    train_steps: int = 20
    warmup_steps: int = 5
    image_size: int = 224
    seq_len: int = 512
    precision: str = "bf16"            # bf16 | fp8 (ResNet conv forward)
    optimizer: str = "momentum"        # momentum | lamb | sgd | adam
    learning_rate: float = 0.1
    decay_steps: int = 0               # 0: constant
    decay_rate: float = 1.0
    staircase: bool = True
    weight_decay: float = 5e-5
    # data-parallel communication (parallel/collective.py, parallel/rccl.py)
    bucket_mb: float = 32.0
    first_bucket_mb: float = 4.0
    compress_bf16: bool = False
    all_reduce_algorithm: str = "allreduce"  # allreduce | hierarchical | reduce_to_one
    collective_engine: str = "auto"          # auto | native | torch
    hipgraph: bool = False
    seed: int = 0
    # session cadence (tf.estimator.RunConfig names)
    checkpoint_dir: Optional[str] = None
    save_checkpoints_secs: Optional[float] = 600.0
    save_checkpoints_steps: Optional[int] = None
    save_summary_steps: int = 100
    log_step_count_steps: int = 100
    keep_checkpoint_max: int = 5
    extra: Dict[str, Any] = field(default_factory=dict)

    _CHOICES = {
        "model": ("resnet50", "bert", "mlp"),
        "precision": ("bf16", "fp8"),
        "optimizer": ("momentum", "lamb", "sgd", "adam"),
        "all_reduce_algorithm": ("allreduce", "hierarchical", "reduce_to_one"),
        "collective_engine": ("auto", "native", "torch"),
    }

    def __post_init__(self):
        self.validate()

    def validate(self):
        for k, allowed in self._CHOICES.items():
            if getattr(self, k) not in allowed:
                raise ValueError("RunConfig.%s = %r (one of %s)" % (k, getattr(self, k), ", ".join(allowed)))
        for k in ("per_replica_batch", "train_steps", "warmup_steps", "decay_steps"):
            if getattr(self, k) < 0:
                raise ValueError("RunConfig.%s must be >= 0" % k)
        if self.bucket_mb <= 0 or self.first_bucket_mb <= 0:
            raise ValueError("bucket sizes must be positive")
        return self

    # ------------------------------------------------------------------ construction
    @classmethod
    def reference_mnist(cls, **kw) -> "RunConfig":
        """The reference script's constants (distribute_training.py:10-17, 22-36, 136-140, 213)."""
        base = dict(model="mlp", per_replica_batch=128, train_steps=10000, warmup_steps=0, optimizer="sgd",
                    learning_rate=0.01, decay_steps=500, decay_rate=0.96, staircase=True, weight_decay=0.0,
                    save_checkpoints_secs=60.0, save_summary_steps=100, log_step_count_steps=100)
        base.update(kw)
        return cls(**base)

    @classmethod
    def fields(cls):
        return [f for f in dataclasses.fields(cls) if f.name != "extra"]

    @classmethod
    def _coerce(cls, name: str, value):
        f = {f.name: f for f in cls.fields()}[name]
        default = f.default
        if value is None or (isinstance(value, str) and value.lower() == "none"):
            return None
        if isinstance(default, bool):
            return value if isinstance(value, bool) else str(value).lower() in ("1", "true", "yes", "on")
        if isinstance(default, int) and not isinstance(default, bool):
            return int(value)
        if isinstance(default, float) or name in ("save_checkpoints_secs",):
            return float(value)
        if name == "save_checkpoints_steps":
            return int(value)
        return value

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RunConfig":
        names = {f.name for f in cls.fields()}
        known = {k: cls._coerce(k, v) for k, v in d.items() if k in names}
        extra = {k: v for k, v in d.items() if k not in names}
        return cls(**known, extra=extra)

    @classmethod
    def from_file(cls, path: str) -> "RunConfig":
        with open(path) as fh:
            if path.endswith((".yaml", ".yml")):
                import yaml
                d = yaml.safe_load(fh) or {}
            else:
                d = json.load(fh)
        return cls.from_dict(d)

    def with_env(self, environ=None) -> "RunConfig":
        """Overrides from TTD_RUN_<FIELD> (e.g. TTD_RUN_BUCKET_MB=64)."""
        env = os.environ if environ is None else environ
        upd = {}
        for f in self.fields():
            v = env.get("TTD_RUN_" + f.name.upper())
            if v is not None:
                upd[f.name] = self._coerce(f.name, v)
        return self.replace(**upd)

    def replace(self, **kw) -> "RunConfig":
        return dataclasses.replace(self, **kw).validate()

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        if not d["extra"]:
            d.pop("extra")
        return d

    # ------------------------------------------------------------------ CLI
    @classmethod
    def add_arguments(cls, parser: argparse.ArgumentParser, prefix: str = "") -> argparse.ArgumentParser:
        """--<field> (dashes) for every field, plus --run-config FILE."""
        parser.add_argument("--%srun-config" % prefix, default=None, help="JSON/YAML RunConfig file")
        for f in cls.fields():
            flag = "--%s%s" % (prefix, f.name.replace("_", "-"))
            if isinstance(f.default, bool):
                parser.add_argument(flag, dest="rc_" + f.name, default=None, nargs="?", const="1",
                                    help="(bool, default %s)" % f.default)
            else:
                kw = {"choices": cls._CHOICES[f.name]} if f.name in cls._CHOICES else {}
                parser.add_argument(flag, dest="rc_" + f.name, default=None, help="(default %s)" % f.default, **kw)
        return parser

    @classmethod
    def from_args(cls, args: argparse.Namespace, prefix: str = "") -> "RunConfig":
        """Defaults <- file (--run-config) <- TTD_RUN_* environment <- explicit flags."""
        path = getattr(args, (prefix + "run_config").replace("-", "_"), None)
        cfg = cls.from_file(path) if path else cls()
        cfg = cfg.with_env()
        upd = {}
        for f in cls.fields():
            v = getattr(args, "rc_" + f.name, None)
            if v is not None:
                upd[f.name] = cls._coerce(f.name, v)
        return cfg.replace(**upd)
