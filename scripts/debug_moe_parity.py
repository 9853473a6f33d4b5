"""Debug helper: per-layer residual comparison CPU vs GPU for the HF-parity Mixtral."""
import os
import pathlib
import sys
import tempfile

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import test_hf_parity as T  # noqa: E402
from p2p_llm_chat_go_amd.models import moe as MOE  # noqa: E402

model, path = T._make(pathlib.Path(tempfile.mkdtemp()), sys.argv[1] if len(sys.argv) > 1 else "mixtral")
rec = {}
orig = MOE.moe_forward


def hooked(m, lw, ws, R):
    key = (m.device.type, len(rec.get(m.device.type, [])))
    before = ws.h[:R].float().cpu().clone()
    orig(m, lw, ws, R)
    rec.setdefault(m.device.type, []).append((before, ws.h[:R].float().cpu().clone(),
                                              ws.moe.topk_ids[:R * 2].cpu().clone(),
                                              ws.moe.cnt.cpu().clone()))


MOE.moe_forward = hooked
for dev in ("cpu", "cuda"):
    eng = T._engine(path, dev)
    pages = [eng.kv.allocator.alloc(2)]
    eng.prefill([[1, 5, 9, 33, 7]], pages, return_logits=True)
for i, (c, g) in enumerate(zip(rec["cpu"], rec["cuda"])):
    print("layer", i, "h_in rel", ((g[0] - c[0]).norm() / c[0].norm()).item(),
          "h_out rel", ((g[1] - c[1]).norm() / c[1].norm()).item(), "nan", bool(g[1].isnan().any()))
    print("  ids cpu", c[2].tolist(), "gpu", g[2].tolist(), "cnt", c[3].tolist(), g[3].tolist())
