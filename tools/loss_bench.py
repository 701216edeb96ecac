"""esgpt_output_loss_ex at a CI config's head layout (LOSS_BENCH_CFG, default C2), per loss-term subset and per
event-kernel path (stream / row-staged / generic): graph-replayed launch time (count + event + reduce kernels).

    python tools/loss_bench.py            LOSS_BENCH_CFG=C5 LOSS_BENCH_B=16 python tools/loss_bench.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import graph_time_ms  # noqa: E402
from eventstreamgpt_amd import _lib as L  # noqa: E402
from eventstreamgpt_amd.kernels import batch_view, err_word  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402
from eventstreamgpt_amd.transformer import model_output as MO  # noqa: E402
from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling  # noqa


def main():
    dev = torch.device("cuda")
    bc = CONFIGS[os.environ.get("LOSS_BENCH_CFG", "C2")]
    model = CIPPTForGenerativeSequenceModeling(bc.model_config())
    bsz = int(os.environ.get("LOSS_BENCH_B", "32"))  # batch size (rows = B * (L + 1): waves per resident round)
    batch = bc.batch(0, batch_size=bsz).to(dev)
    layer = model.output_layer
    layer._layout = layer._build_layout()
    terms, _ = layer._terms_for(MO.all_classification_measurements(layer),
                                MO.all_regression_measurements(layer.config), 0)
    tte = layer._tte_spec(layer._layout["n_content"])
    lib = L.load()
    bv = batch_view(batch)
    B, Lq, M = bv.B, bv.L, bv.M
    C = layer._layout["n_content"] + tte.K * (1 if tte.kind == L.TTE_EXP else 3)
    C += (-C) % 8
    g = torch.Generator(device=dev).manual_seed(4)
    zc = torch.randn(B * Lq, C, device=dev, generator=g).bfloat16()
    bias = torch.zeros(C, device=dev).bfloat16()
    dzc = torch.empty_like(zc)
    dbias = torch.empty(B, C, device=dev)
    losses = torch.empty(len(terms) + 2, device=dev)
    err = err_word(dev)
    kinds = {L.TERM_SINGLE: "single", L.TERM_MULTI: "multi", L.TERM_MVREG: "mvreg", L.TERM_UVREG: "uvreg"}
    print(json.dumps({"B": B, "L": Lq, "M": M, "C": C,
                      "terms": [(kinds[t.kind], t.vocab_end - t.vocab_start) for t in terms]}))

    def launcher(sub, path=L.LOSS_PATH_AUTO):
        arr = (L.EsgptLossTerm * max(1, len(sub)))(*sub)
        nb = lib.esgpt_output_loss_workspace(B, Lq, len(sub))
        ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)

        def fwd():
            L.check(lib.esgpt_output_loss_ex(bv.ref, zc.data_ptr(), C, 1, 1, bias.data_ptr(), zc.data_ptr(), C,
                                             L.BF16, arr, len(sub), ctypes.byref(tte), dzc.data_ptr(), dzc.data_ptr(),
                                             dbias.data_ptr(), losses[: len(sub) + 2].data_ptr(), ws.data_ptr(), nb,
                                             err.data_ptr(), path, L.stream()), "output_loss")
        return fwd, (arr, ws)

    if "--pmc" in sys.argv:  # eager launches of a term subset (counter collection): --pmc [all | i]
        k = sys.argv[sys.argv.index("--pmc") + 1] if len(sys.argv) > sys.argv.index("--pmc") + 1 else "all"
        fn, keep = launcher(list(terms) if k == "all" else [terms[int(k)]])
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        err.zero_()
        return
    subsets = {"all": list(terms)}
    if os.environ.get("LOSS_BENCH_ONLY") != "all":
        for i, t in enumerate(terms):
            subsets[f"only_{i}_{kinds[t.kind]}"] = [t]
    algo = B * Lq * C * 4 + B * Lq * M * 21
    paths = ((L.LOSS_PATH_STREAM, "stream"), (L.LOSS_PATH_ROW_STAGED, "row_staged"), (L.LOSS_PATH_GENERIC, "generic"))
    if os.environ.get("LOSS_BENCH_ONLY") == "all":
        paths = paths[:1]
    for path, pname in paths:
        for name, sub in subsets.items():
            fn, keep = launcher(sub, path)
            try:
                us = graph_time_ms(fn) * 1e3
            except RuntimeError as e:  # a forced path that does not apply to this layout
                print(json.dumps({"path": pname, "terms": name, "error": str(e)[:80]}))
                break
            rec = {"path": pname, "terms": name, "us": round(us, 2)}
            if name == "all":
                rec["losses"] = [round(x, 6) for x in losses[: len(sub) + 2].tolist()]
                rec["dz_sum"] = round(float(dzc.float().sum()), 6)
                rec["algorithmic_MB"] = round(algo / 1e6, 2)
                rec["TB_s"] = round(algo / us / 1e6, 3)
            print(json.dumps(rec))
    err.zero_()


if __name__ == "__main__":
    main()
