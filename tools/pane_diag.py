"""Step-by-step run of the heavy-disorder sliding parity case, printing progress (pane-mode diagnosis)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import _stream, _gpu_op
import torch
cfg = dict(assigner="sliding", size=3000, slide=1000)
batches, wms = _stream(120_000, 10_000, 5000, bound=400, jitter=1500, rate=100_000)
op = _gpu_op(**cfg)
for i, ((k, t, v), wm) in enumerate(zip(batches, wms)):
    print("step", i, "push", len(k), flush=True)
    op.process(k, t, v)
    print("  stats", op.stats(), flush=True)
    print("  watermark", wm, flush=True)
    op.watermark(wm)
    print("  rows", len(op.rows()), flush=True)
print("done", flush=True)
