"""The §8(d) C5 embed-bag microbench (bench.py _c5_embed_bf16_microbench: 2 GiB bf16 table, uniform indices) timed
with the input-layer flag variants, to separate the row gathers from the per-event time prefix and static rows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from eventstreamgpt_amd import _lib as L  # noqa: E402
from eventstreamgpt_amd.kernels import batch_view, err_word  # noqa: E402

dev = torch.device("cuda")
fwd, nbytes, nnz, (table, out, batch, div, times) = bench._c5_embed_bf16_microbench(dev)
lib = L.load()
bv = batch_view(batch)
err = err_word(dev)
V, D = table.shape
for name, flags in [("static|time", L.EMB_STATIC | L.EMB_TIME), ("static", L.EMB_STATIC), ("time", L.EMB_TIME),
                    ("none", 0)]:
    def fn(flags=flags):
        L.check(lib.esgpt_embed_joint_fwd_ex(bv.ref, None, table.data_ptr(), L.BF16, V, D, div.data_ptr(),
                                             div.data_ptr(), flags, 0.5, 0.5, out.data_ptr(), err.data_ptr(),
                                             L.stream()), "embed")
    ms = bench.graph_time_ms(fn)
    print(f"{name:12s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:8.3f} TB/s per occurrence", flush=True)
ms = bench.graph_time_ms(fwd)
print(f"op form (event times + bag kernel, static|time) {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:8.3f} TB/s per occurrence")

