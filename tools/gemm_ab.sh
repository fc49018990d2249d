#!/bin/bash
# GEMM A/B on BERT-Large b128 shapes: big256 8-wave vs TTD_BIG_PP=1 vs torch (hipBLASLt)
for shp in "65536 4096 1024 0 1" "65536 1024 4096 0 1" "65536 3072 1024 0 1" "4096 1024 65536 1 0" "65536 1024 4096 0 0"; do
  timeout -k 5 60 python3 tools/one_gemm.py $shp 20 || exit 1
  TTD_BIG_PP=1 timeout -k 5 60 python3 tools/one_gemm.py $shp 20 || exit 1
done
timeout -k 5 60 python3 - <<'PY'
import torch, time
for M, N, K in ((65536, 4096, 1024), (65536, 1024, 4096), (65536, 3072, 1024)):
    a = torch.randn(M, K, device="cuda").bfloat16(); b = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(3): c = a @ b.t()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(20): c = a @ b.t()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20
    print("torch M=%d N=%d K=%d: %.1f us %.0f TF/s" % (M, N, K, dt * 1e6, 2 * M * N * K / dt / 1e12))
PY
