"""Checkpoints in the TensorFlow on-disk formats.

* TensorBundle V2 (`<prefix>.index` LevelDB table + `<prefix>.data-XXXXX-of-YYYYY`) via the
  native writer/reader/merger (csrc/runtime/bundle.cc);
* the directory's `checkpoint` state file (CheckpointState text proto);
* `Saver` — name-based keys (`hidden1/kernel`, ..., `global_step`), max_to_keep pruning, as
  installed by MonitoredTrainingSession's CheckpointSaverHook in the reference
  (/root/reference/distribute_training.py:204-215, save_checkpoint_secs=60);
* `Checkpoint` / `CheckpointManager` — object-based tf.train.Checkpoint keys
  (`model/<var>/.ATTRIBUTES/VARIABLE_VALUE`, optimizer slots under `.OPTIMIZER_SLOT`,
  `save_counter`) plus the `_CHECKPOINTABLE_OBJECT_GRAPH` TrackableObjectGraph proto.

Variables are exported in TF layout: our conv kernels are stored [K,R,S,C] (implicit-GEMM B
operand) and become TF's [R,S,C,K] here (ParamSpec.meta["layout"] == "KRSC").
"""
from __future__ import annotations

import ctypes
import glob
import os
import re
import shutil
import time
import uuid
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from .. import _native
from ..utils import proto

# TF DataType enum
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8, DT_INT16, DT_INT8, DT_STRING, DT_INT64, DT_BOOL = 1, 2, 3, 4, 5, 6, 7, 9, 10
DT_BFLOAT16, DT_HALF = 14, 19

_NP2DT = {np.dtype("float32"): DT_FLOAT, np.dtype("float64"): DT_DOUBLE, np.dtype("int32"): DT_INT32,
          np.dtype("uint8"): DT_UINT8, np.dtype("int16"): DT_INT16, np.dtype("int8"): DT_INT8,
          np.dtype("int64"): DT_INT64, np.dtype("bool"): DT_BOOL, np.dtype("float16"): DT_HALF}
_DT2NP = {v: k for k, v in _NP2DT.items()}

OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"


def _lib():
    lib = _native.rt()
    if not getattr(lib, "_bundle_sigs", False):
        vp, cp, ci = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int
        lib.ttd_bundle_writer_open.restype = vp
        lib.ttd_bundle_writer_open.argtypes = [cp, ci, ci]
        lib.ttd_bundle_writer_add.argtypes = [vp, cp, ci, ci, ctypes.POINTER(ctypes.c_int64), vp, ctypes.c_uint64]
        lib.ttd_bundle_writer_add_strings.argtypes = [vp, cp, ci, ctypes.POINTER(ctypes.c_int64), ci,
                                                      ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64)]
        lib.ttd_bundle_writer_finish.argtypes = [vp]
        lib.ttd_bundle_merge.argtypes = [ci, ctypes.POINTER(ctypes.c_char_p), cp]
        lib.ttd_bundle_reader_open.restype = vp
        lib.ttd_bundle_reader_open.argtypes = [cp]
        lib.ttd_bundle_reader_num_entries.argtypes = [vp]
        lib.ttd_bundle_reader_num_shards.argtypes = [vp]
        lib.ttd_bundle_reader_key.restype = cp
        lib.ttd_bundle_reader_key.argtypes = [vp, ci]
        lib.ttd_bundle_reader_entry.argtypes = [vp, cp, ctypes.POINTER(ci), ctypes.POINTER(ctypes.c_int64),
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ci),
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]
        lib.ttd_bundle_reader_read.argtypes = [vp, cp, vp, ctypes.c_uint64]
        lib.ttd_bundle_reader_close.argtypes = [vp]
        lib._bundle_sigs = True
    return lib


class CheckpointError(IOError):
    pass


def _err():
    return CheckpointError(_native.rt_error())


def _to_numpy(v) -> Tuple[np.ndarray, int]:
    """-> (contiguous little-endian array, TF dtype)."""
    if isinstance(v, torch.Tensor):
        t = v.detach()
        if t.dtype == torch.bfloat16:
            return t.cpu().contiguous().view(torch.int16).numpy().view(np.uint16), DT_BFLOAT16
        a = t.cpu().contiguous().numpy()
    else:
        a = np.asarray(v)
    if not a.flags["C_CONTIGUOUS"]:
        a = a.copy(order="C")  # (np.ascontiguousarray would turn 0-d scalars into shape [1])
    if a.dtype not in _NP2DT:
        raise TypeError("unsupported checkpoint dtype %s" % a.dtype)
    return a, _NP2DT[a.dtype]


class BundleWriter:
    def __init__(self, prefix: str, shard_id: int = 0, num_shards: int = 1):
        d = os.path.dirname(prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        self._h = _lib().ttd_bundle_writer_open(prefix.encode(), shard_id, num_shards)
        if not self._h:
            raise _err()
        self.prefix = prefix

    def add(self, key: str, value, dtype: Optional[int] = None):
        a, dt = _to_numpy(value)
        if dtype is not None:
            dt = dtype
        shape = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
        if _lib().ttd_bundle_writer_add(self._h, key.encode(), dt, a.ndim, shape, a.ctypes.data, a.nbytes) != 0:
            raise _err()

    def add_strings(self, key: str, values: List[bytes], shape=None):
        shape = tuple(shape) if shape is not None else (() if len(values) == 1 else (len(values),))
        cshape = (ctypes.c_int64 * max(1, len(shape)))(*shape)
        arr = (ctypes.c_char_p * len(values))(*values)
        lens = (ctypes.c_uint64 * len(values))(*[len(v) for v in values])
        if _lib().ttd_bundle_writer_add_strings(self._h, key.encode(), len(shape), cshape, len(values), arr, lens) != 0:
            raise _err()

    def finish(self):
        if _lib().ttd_bundle_writer_finish(self._h) != 0:
            self._h = None
            raise _err()
        self._h = None


def merge_bundles(in_prefixes: List[str], out_prefix: str):
    arr = (ctypes.c_char_p * len(in_prefixes))(*[p.encode() for p in in_prefixes])
    if _lib().ttd_bundle_merge(len(in_prefixes), arr, out_prefix.encode()) != 0:
        raise _err()


class BundleReader:
    def __init__(self, prefix: str):
        self._h = _lib().ttd_bundle_reader_open(prefix.encode())
        if not self._h:
            raise _err()
        self.prefix = prefix

    def keys(self) -> List[str]:
        lib = _lib()
        return [lib.ttd_bundle_reader_key(self._h, i).decode() for i in range(lib.ttd_bundle_reader_num_entries(self._h))]

    @property
    def num_shards(self):
        return _lib().ttd_bundle_reader_num_shards(self._h)

    def entry(self, key: str) -> dict:
        dt = ctypes.c_int()
        shape = (ctypes.c_int64 * 32)()
        nb = ctypes.c_uint64()
        shard = ctypes.c_int()
        off = ctypes.c_uint64()
        crc = ctypes.c_uint32()
        nd = _lib().ttd_bundle_reader_entry(self._h, key.encode(), ctypes.byref(dt), shape, ctypes.byref(nb),
                                            ctypes.byref(shard), ctypes.byref(off), ctypes.byref(crc))
        if nd < 0:
            raise KeyError(key)
        return {"dtype": dt.value, "shape": tuple(shape[i] for i in range(nd)), "size": nb.value,
                "shard_id": shard.value, "offset": off.value, "crc32c": crc.value}

    def read_raw(self, key: str) -> bytes:
        e = self.entry(key)
        buf = ctypes.create_string_buffer(max(1, e["size"]))
        rc = _lib().ttd_bundle_reader_read(self._h, key.encode(), buf, e["size"])
        if rc != 0:
            raise _err()
        return buf.raw[:e["size"]]

    def read(self, key: str):
        e = self.entry(key)
        raw = self.read_raw(key)
        if e["dtype"] == DT_STRING:
            return _decode_strings(raw, int(np.prod(e["shape"])) if e["shape"] else 1)
        if e["dtype"] == DT_BFLOAT16:
            a = np.frombuffer(raw, dtype=np.uint16).copy().reshape(e["shape"])
            return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16)
        return np.frombuffer(raw, dtype=_DT2NP[e["dtype"]]).copy().reshape(e["shape"])

    def close(self):
        if self._h:
            _lib().ttd_bundle_reader_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _decode_strings(raw: bytes, n: int) -> List[bytes]:
    lens, i = [], 0
    for _ in range(n):
        v, sh = 0, 0
        while True:
            b = raw[i]
            i += 1
            v |= (b & 0x7F) << sh
            if not b & 0x80:
                break
            sh += 7
        lens.append(v)
    i += 4  # masked crc32c of the lengths (verified by the native reader's whole-entry crc)
    out = []
    for n_ in lens:
        out.append(raw[i:i + n_])
        i += n_
    return out


# ------------------------------------------------------------------ checkpoint state file
def _quote(s):
    return '"%s"' % s.replace("\\", "\\\\").replace('"', '\\"')


def update_checkpoint_state(directory: str, model_checkpoint_path: str, all_model_checkpoint_paths: List[str],
                            all_timestamps: Optional[List[float]] = None, latest_filename: str = "checkpoint"):
    """Writes the CheckpointState text proto (paths relative to `directory` when inside it)."""
    def rel(p):
        return os.path.relpath(p, directory) if os.path.dirname(os.path.abspath(p)) == os.path.abspath(directory) else p
    lines = ["model_checkpoint_path: %s" % _quote(rel(model_checkpoint_path))]
    for p in all_model_checkpoint_paths:
        lines.append("all_model_checkpoint_paths: %s" % _quote(rel(p)))
    for t in all_timestamps or []:
        lines.append("all_model_checkpoint_timestamps: %.6f" % t)
    if all_timestamps:
        lines.append("last_preserved_timestamp: %.6f" % min(all_timestamps))
    tmp = os.path.join(directory, ".%s.tmp%s" % (latest_filename, uuid.uuid4().hex[:8]))
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(directory, latest_filename))


def get_checkpoint_state(directory: str, latest_filename: str = "checkpoint") -> Optional[dict]:
    path = os.path.join(directory, latest_filename)
    if not os.path.exists(path):
        return None
    st = {"model_checkpoint_path": None, "all_model_checkpoint_paths": [], "all_model_checkpoint_timestamps": []}
    for line in open(path):
        m = re.match(r'\s*(\w+)\s*:\s*(.*)$', line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if v.startswith('"'):
            v = v[1:-1].replace('\\"', '"').replace("\\\\", "\\")
            if not os.path.isabs(v):
                v = os.path.join(directory, v)
        if k == "model_checkpoint_path":
            st[k] = v
        elif k == "all_model_checkpoint_paths":
            st[k].append(v)
        elif k == "all_model_checkpoint_timestamps":
            st[k].append(float(v))
    return st


def checkpoint_exists(prefix: str) -> bool:
    return os.path.exists(prefix + ".index")


def latest_checkpoint(directory: str, latest_filename: str = "checkpoint") -> Optional[str]:
    st = get_checkpoint_state(directory, latest_filename)
    if st and st["model_checkpoint_path"] and checkpoint_exists(st["model_checkpoint_path"]):
        return st["model_checkpoint_path"]
    return None


def remove_checkpoint(prefix: str):
    for f in glob.glob(glob.escape(prefix) + ".index") + glob.glob(glob.escape(prefix) + ".data-*") + \
            glob.glob(glob.escape(prefix) + ".meta"):
        try:
            os.remove(f)
        except OSError:
            pass


def list_variables(ckpt: str) -> List[Tuple[str, tuple]]:
    """tf.train.list_variables: (name, shape) of every tensor in a checkpoint (or dir)."""
    if os.path.isdir(ckpt):
        ckpt = latest_checkpoint(ckpt)
    r = BundleReader(ckpt)
    try:
        return [(k, r.entry(k)["shape"]) for k in r.keys()]
    finally:
        r.close()


def load_variable(ckpt: str, name: str):
    if os.path.isdir(ckpt):
        ckpt = latest_checkpoint(ckpt)
    r = BundleReader(ckpt)
    try:
        return r.read(name)
    finally:
        r.close()


# ------------------------------------------------------------------ TF-layout variable export
def export_value(spec, t: torch.Tensor) -> np.ndarray:
    a = t.detach().float().cpu().numpy() if t.dtype != torch.int64 else t.detach().cpu().numpy()
    lay = spec.meta.get("layout") if spec is not None else None
    if lay == "KRSC":
        cin = spec.meta.get("cin", a.shape[-1])
        a = a[..., :cin].transpose(1, 2, 3, 0).copy(order="C")  # -> [R,S,C,K]
    elif lay == "NK":  # dense kernel stored [out, in] (GEMM B operand) -> TF [in, out]
        a = a.T.copy(order="C")
    if spec is not None and "rows" in spec.meta:  # padded leading dim (e.g. vocabulary to a multiple of 64)
        a = a[:spec.meta["rows"]].copy(order="C")
    return a if a.flags["C_CONTIGUOUS"] else a.copy(order="C")


def import_value(spec, a: np.ndarray, target: torch.Tensor):
    a = np.asarray(a)
    lay = spec.meta.get("layout") if spec is not None else None
    if lay == "KRSC":
        w = np.zeros(tuple(target.shape), dtype=np.float32)
        cin = a.shape[2]
        w[..., :cin] = a.transpose(3, 0, 1, 2)
        a = w
    elif lay == "NK":
        a = a.T
    if spec is not None and "rows" in spec.meta and a.shape[0] != target.shape[0]:
        w = np.zeros(tuple(target.shape), dtype=np.float32)
        w[:a.shape[0]] = a
        a = w
    with torch.no_grad():
        target.copy_(torch.from_numpy(np.ascontiguousarray(a)).reshape(target.shape).to(target.dtype))


# ------------------------------------------------------------------ name-based Saver
class Saver:
    """tf.train.Saver (V2, name-based keys).

    var_list: a FlatParams (all its variables), a dict name -> tensor, or a list of
    (name, getter, setter) providers; `extra` adds e.g. {"global_step": callable}.
    sharded=True with `shard_writers` lets each parameter-server task write its own shard
    which the chief merges (MergeV2Checkpoints).
    """

    def __init__(self, var_list=None, max_to_keep: int = 5, keep_checkpoint_every_n_hours: float = 10000.0,
                 extra: Optional[dict] = None, latest_filename: str = "checkpoint", on_restore=None):
        self.var_list = var_list
        self.max_to_keep = max_to_keep
        self.extra = extra or {}
        # called after every restore: e.g. FlatParams.refresh_compute, so the bf16 compute
        # copy the GPU engines run on follows the restored fp32 master weights
        self.on_restore = list(on_restore or [])
        self.latest_filename = latest_filename
        self._last: List[Tuple[str, float]] = []

    def _items(self):
        from .flat import FlatParams
        vl = self.var_list
        if isinstance(vl, FlatParams):
            for s in vl.specs:
                yield s.name, (lambda s=s: export_value(s, vl.var[s.name])), \
                    (lambda a, s=s: import_value(s, a, vl.var[s.name]))
            return
        if isinstance(vl, dict):
            for k, t in vl.items():
                yield k, (lambda t=t: export_value(None, t)), (lambda a, t=t: import_value(None, a, t))
            return
        for item in vl or []:
            yield item

    def save(self, sess=None, save_path: str = "model.ckpt", global_step=None, write_state: bool = True,
             shard_writers=None) -> str:
        step = int(global_step) if global_step is not None else None
        prefix = "%s-%d" % (save_path, step) if step is not None else save_path
        d = os.path.dirname(prefix) or "."
        os.makedirs(d, exist_ok=True)
        if shard_writers:
            # every shard writer writes a single-shard bundle into a temp dir; the chief merges.
            tmpdir = prefix + "_temp_" + uuid.uuid4().hex
            os.makedirs(tmpdir)
            parts = []
            for k, w in enumerate(shard_writers):
                p = os.path.join(tmpdir, "part-%05d" % k)
                w(p)
                parts.append(p)
            merge_bundles(parts, prefix)
            shutil.rmtree(tmpdir, ignore_errors=True)
        else:
            w = BundleWriter(prefix)
            for name, get, _ in self._items():
                w.add(name, get())
            for name, get in self.extra.items():
                w.add(name, np.asarray(get()))
            w.finish()
        if write_state:
            self._last = [(p, t) for p, t in self._last if p != prefix] + [(prefix, time.time())]
            while len(self._last) > self.max_to_keep > 0:
                old, _ = self._last.pop(0)
                remove_checkpoint(old)
            update_checkpoint_state(d, prefix, [p for p, _ in self._last], [t for _, t in self._last],
                                    self.latest_filename)
        return prefix

    def restore(self, sess=None, save_path: str = None, strict: bool = True):
        r = BundleReader(save_path)
        try:
            keys = set(r.keys())
            for name, _, set_ in self._items():
                if name in keys:
                    set_(r.read(name))
                elif strict:
                    raise CheckpointError("variable %s not found in %s" % (name, save_path))
            out = {}
            for name in self.extra:
                if name in keys:
                    out[name] = r.read(name)
        finally:
            r.close()
        from .flat import FlatParams
        if isinstance(self.var_list, FlatParams):
            self.var_list.refresh_compute()
        for fn in self.on_restore:
            fn()
        return out

    def recover_last_checkpoints(self, paths: List[str]):
        self._last = [(p, time.time()) for p in paths if checkpoint_exists(p)]


# ------------------------------------------------------------------ object-based Checkpoint
class _Node:
    def __init__(self):
        self.children: List[Tuple[str, "_Node"]] = []
        self.attr = None  # (full_name, key, getter, setter)
        self.slots: List[Tuple["_Node", str, "_Node"]] = []
        self.id = -1


def _encode_object_graph(nodes: List[_Node]) -> bytes:
    out = b""
    for n in nodes:
        body = b""
        for name, ch in n.children:
            body += proto.f_msg(1, proto.f_varint(1, ch.id) + proto.f_str(2, name))
        if n.attr is not None:
            full, key = n.attr[0], n.attr[1]
            body += proto.f_msg(2, proto.f_str(1, "VARIABLE_VALUE") + proto.f_str(2, full) + proto.f_str(3, key))
        for orig, slot_name, slot_node in n.slots:
            body += proto.f_msg(3, proto.f_varint(1, orig.id) + proto.f_str(2, slot_name) +
                                proto.f_varint(3, slot_node.id))
        out += proto.f_msg(1, body)
    return out


def decode_object_graph(buf: bytes) -> List[dict]:
    nodes = []
    for nb in proto.decode(buf).get(1, []):
        d = proto.decode(nb)
        node = {"children": [], "attributes": [], "slot_variables": []}
        for c in d.get(1, []):
            cd = proto.decode(c)
            node["children"].append((cd.get(1, [0])[0], cd[2][0].decode() if 2 in cd else ""))
        for a in d.get(2, []):
            ad = proto.decode(a)
            node["attributes"].append({k: ad[f][0].decode() for k, f in (("name", 1), ("full_name", 2),
                                                                         ("checkpoint_key", 3)) if f in ad})
        for sv in d.get(3, []):
            sd = proto.decode(sv)
            node["slot_variables"].append((sd.get(1, [0])[0], sd[2][0].decode(), sd.get(3, [0])[0]))
        nodes.append(node)
    return nodes


class Checkpoint:
    """tf.train.Checkpoint over framework objects.

    Accepted attributes: FlatParams, objects exposing `.params` (models), flat optimizers
    (their slot buffers become `.OPTIMIZER_SLOT` entries of each variable), torch tensors and
    objects with `.numpy()`/`.assign()` (e.g. GlobalStep).
    """

    def __init__(self, **kwargs):
        self._objs = dict(kwargs)
        self.save_counter = 0

    # -- graph construction
    def _build(self):
        from .flat import FlatParams, FlatOptimizer
        root = _Node()
        nodes = [root]
        var_nodes = {}

        def add(parent, name):
            n = _Node()
            n.id = len(nodes)
            nodes.append(n)
            parent.children.append((name, n))
            return n

        def node_for_path(parent, path, cache):
            cur, acc = parent, []
            for comp in path.split("/"):
                acc.append(comp)
                key = "/".join(acc)
                if key not in cache:
                    cache[key] = add(cur, comp)
                cur = cache[key]
            return cur

        def flat_of(o):
            if isinstance(o, FlatParams):
                return o
            p = getattr(o, "params", None)
            return p if isinstance(p, FlatParams) else None

        optimizers = []
        for attr, obj in self._objs.items():
            fp = flat_of(obj)
            if fp is not None:
                cache = {}
                top = add(root, attr)
                for s in fp.specs:
                    leaf = node_for_path(top, s.name, cache)
                    key = "%s/%s/.ATTRIBUTES/VARIABLE_VALUE" % (attr, s.name)
                    leaf.attr = (s.name, key, (lambda s=s, fp=fp: export_value(s, fp.var[s.name])),
                                 (lambda a, s=s, fp=fp: import_value(s, a, fp.var[s.name])))
                    var_nodes[(id(fp), s.name)] = (attr, leaf, s)
            elif isinstance(obj, FlatOptimizer):
                optimizers.append((attr, obj))
            else:
                n = add(root, attr)
                key = "%s/.ATTRIBUTES/VARIABLE_VALUE" % attr
                n.attr = (attr, key, (lambda o=obj: _value_of(o)), (lambda a, o=obj: _assign(o, a)))
        for attr, opt in optimizers:
            onode = add(root, attr)
            it = add(onode, "iter")
            it.attr = ("iter", "%s/iter/.ATTRIBUTES/VARIABLE_VALUE" % attr,
                       (lambda o=opt: np.asarray(o._host_step, dtype=np.int64)),
                       (lambda a, o=opt: o.set_step(int(np.asarray(a)))))
            fp = opt.p
            for slot_name, buf in _slots(opt):
                for s in fp.specs:
                    if not s.trainable or (id(fp), s.name) not in var_nodes:
                        continue
                    vattr, vnode, spec = var_nodes[(id(fp), s.name)]
                    sn = _Node()
                    sn.id = len(nodes)
                    nodes.append(sn)
                    o, n = fp.offsets[s.name], int(np.prod(s.shape))
                    view = buf[o:o + n].view(tuple(s.shape))
                    key = "%s/%s/.OPTIMIZER_SLOT/%s/%s/.ATTRIBUTES/VARIABLE_VALUE" % (vattr, s.name, attr, slot_name)
                    sn.attr = ("%s/%s" % (s.name, slot_name), key, (lambda s=s, v=view: export_value(s, v)),
                               (lambda a, s=s, v=view: import_value(s, a, v)))
                    onode.slots.append((vnode, slot_name, sn))
        sc = add(root, "save_counter")
        sc.attr = ("save_counter", "save_counter/.ATTRIBUTES/VARIABLE_VALUE",
                   lambda: np.asarray(self.save_counter, dtype=np.int64),
                   lambda a: setattr(self, "save_counter", int(np.asarray(a))))
        return nodes

    def write(self, file_prefix: str) -> str:
        nodes = self._build()
        w = BundleWriter(file_prefix)
        for n in nodes:
            if n.attr is not None:
                w.add(n.attr[1], n.attr[2]())
        w.add_strings(OBJECT_GRAPH_KEY, [_encode_object_graph(nodes)])
        w.finish()
        return file_prefix

    def save(self, file_prefix: str) -> str:
        self.save_counter += 1
        prefix = "%s-%d" % (file_prefix, self.save_counter)
        self.write(prefix)
        d = os.path.dirname(prefix) or "."
        st = get_checkpoint_state(d)
        paths = (st["all_model_checkpoint_paths"] if st else []) + [prefix]
        update_checkpoint_state(d, prefix, paths)
        return prefix

    def restore(self, save_path: str, strict: bool = False):
        if save_path is None:
            return self
        if os.path.isdir(save_path):
            save_path = latest_checkpoint(save_path)
        r = BundleReader(save_path)
        try:
            keys = set(r.keys())
            missing = []
            for n in self._build():
                if n.attr is None:
                    continue
                if n.attr[1] in keys:
                    n.attr[3](r.read(n.attr[1]))
                else:
                    missing.append(n.attr[1])
            if strict and missing:
                raise CheckpointError("missing keys: %s" % missing[:5])
        finally:
            r.close()
        for fp in self._flat_params():  # the bf16 compute copies follow the restored masters
            fp.refresh_compute()
        return self

    read = restore

    def _flat_params(self):
        from .flat import FlatParams, FlatOptimizer
        out = []
        for obj in self._objs.values():
            fp = obj if isinstance(obj, FlatParams) else getattr(obj, "params", None)
            if isinstance(obj, FlatOptimizer):
                fp = obj.p
            if isinstance(fp, FlatParams) and all(fp is not o for o in out):
                out.append(fp)
        return out


def _slots(opt):
    out = []
    for name in ("mom", "m", "v"):
        buf = getattr(opt, name, None)
        if isinstance(buf, torch.Tensor):
            out.append(({"mom": "momentum", "m": "m", "v": "v"}[name], buf))
    return out


def _value_of(o):
    if isinstance(o, torch.Tensor):
        return o.detach().cpu().numpy()
    if hasattr(o, "numpy"):
        return np.asarray(o.numpy())
    return np.asarray(o)


def _assign(o, a):
    if isinstance(o, torch.Tensor):
        with torch.no_grad():
            o.copy_(torch.as_tensor(np.asarray(a)).reshape(o.shape))
    elif hasattr(o, "assign"):
        o.assign(a)
    else:
        raise TypeError("cannot restore into %r" % (o,))


class CheckpointManager:
    """tf.train.CheckpointManager: numbered saves `<directory>/ckpt-N`, max_to_keep pruning,
    `checkpoint` state file, latest_checkpoint."""

    def __init__(self, checkpoint: Checkpoint, directory: str, max_to_keep: int = 5, checkpoint_name: str = "ckpt"):
        self.checkpoint = checkpoint
        self.directory = directory
        self.max_to_keep = max_to_keep
        self.prefix = os.path.join(directory, checkpoint_name)
        os.makedirs(directory, exist_ok=True)
        st = get_checkpoint_state(directory)
        self._ckpts = [p for p in (st["all_model_checkpoint_paths"] if st else []) if checkpoint_exists(p)]

    @property
    def latest_checkpoint(self):
        return self._ckpts[-1] if self._ckpts else None

    @property
    def checkpoints(self):
        return list(self._ckpts)

    def save(self, checkpoint_number: Optional[int] = None) -> str:
        if checkpoint_number is None:
            self.checkpoint.save_counter += 1
            n = self.checkpoint.save_counter
        else:
            n = int(checkpoint_number)
            self.checkpoint.save_counter += 1
        path = "%s-%d" % (self.prefix, n)
        self.checkpoint.write(path)
        self._ckpts = [p for p in self._ckpts if p != path] + [path]
        while self.max_to_keep and len(self._ckpts) > self.max_to_keep:
            remove_checkpoint(self._ckpts.pop(0))
        update_checkpoint_state(self.directory, path, self._ckpts)
        return path

    def restore_or_initialize(self):
        if self.latest_checkpoint:
            self.checkpoint.restore(self.latest_checkpoint)
            return self.latest_checkpoint
        return None
