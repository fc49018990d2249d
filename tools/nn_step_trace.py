#!/usr/bin/env python3
"""Which GPU kernels does a `ttd.layers` Sequential training step launch?

    rocprofv3 --kernel-trace --output-format csv -d <dir> -o run -- python3 tools/nn_step_trace.py run
    python3 tools/nn_step_trace.py check <dir>/run_kernel_trace.csv

`run` builds two Sequential models on fp32 GPU tensors — an image head (MaxPooling2D 'SAME',
BatchNormalization, GlobalAveragePooling2D, Dense relu, Dropout, LayerNormalization (width 64,
not one of the fused BERT widths), Dense tanh, Dense) and a text head (Embedding, Flatten,
Dense) — does one untraced warm-up step, then brackets STEPS training steps (GradientTape ->
tf.reduce_mean(sparse softmax xent) -> Optimizer.apply_gradients) with trace-marker kernels.
`check` lists the kernels dispatched between the markers and fails if any is a PyTorch
`at::native` kernel (i.e. an op that silently fell back to torch compute).
"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STEPS = 2


def run():
    import torch

    import tensorflow_train_distributed_amd as ttd
    from tensorflow_train_distributed_amd.ops import kernels as K
    L, N = ttd.layers, ttd.nn
    L.reset_naming(0)
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    img = L.Sequential([L.MaxPooling2D(3, 2, "SAME"), L.BatchNormalization(), L.GlobalAveragePooling2D(),
                        L.Dense(64, "relu"), L.Dropout(0.1), L.LayerNormalization(), L.Dense(32, "tanh"),
                        L.Dense(10)])
    txt = L.Sequential([L.Embedding(50, 24), L.Flatten(), L.Dense(10)])
    x = torch.randn(16, 9, 9, 12, generator=g).to(dev)
    ids = torch.randint(0, 50, (16, 6), generator=g).to(dev)
    y = torch.randint(0, 10, (16,), generator=g).to(dev)
    models = [(img, x, ttd.train.GradientDescentOptimizer(0.1)), (txt, ids, ttd.train.AdamOptimizer(1e-3))]
    for m, inp, _ in models:
        m(inp)
        m.to_flat(dev)

    def step():
        out = []
        for m, inp, opt in models:
            with ttd.GradientTape() as tape:
                logits = m(inp)
                loss = ttd.reduce_mean(N.sparse_softmax_cross_entropy_with_logits(labels=y, logits=logits))
            tv = m.trainable_variables
            grads = tape.gradient(loss, tv)
            opt.apply_gradients(zip(grads, tv))
            out.append(loss)
        return out

    first = [float(v) for v in step()]  # warm-up: optimizer slots, seeds, chunk tables
    torch.cuda.synchronize()
    K.trace_marker(1)
    for _ in range(STEPS):
        last = step()
    K.trace_marker(2)
    torch.cuda.synchronize()
    last = [float(v) for v in last]
    print("losses first %s last %s" % (first, last), flush=True)


def kernels_between_markers(path):
    with open(path) as f:
        rows = list(csv.DictReader(f))
    key = "Start_Timestamp" if rows and "Start_Timestamp" in rows[0] else None
    if key:
        rows.sort(key=lambda r: int(r[key]))
    name_col = "Kernel_Name"
    idx = [i for i, r in enumerate(rows) if "trace_marker_kernel" in r[name_col]]
    if len(idx) < 2:
        raise SystemExit("trace markers not found in %s" % path)
    return [r[name_col] for r in rows[idx[0] + 1:idx[-1]]]


def check(path):
    names = kernels_between_markers(path)
    counts = collections.Counter(names)
    bad = {n: c for n, c in counts.items() if "at::native" in n or "at::cuda" in n}
    for n, c in counts.most_common():
        print("%4d  %s%s" % (c, "TORCH " if n in bad else "", n[:160]))
    print("%d kernels per %d steps, %d distinct, %d torch-native" % (len(names), STEPS, len(counts), len(bad)))
    return 1 if bad or not names else 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        sys.exit(check(sys.argv[2]))
