"""engine.cluster on the GPU box: the node's multi-GPU serving path with one rank
process per GPU (here the box's single MI355X, ENGINE_CLUSTER=1 semantics):
spawned before this process touches the GPU, replies equal the in-process
engine's."""
import json

import pytest

pytestmark = pytest.mark.gpu


def test_cluster_one_gpu_matches_in_process():
    from p2p_llm_chat_go_amd.engine.cluster import ClusterServer

    req = json.dumps({"model": "llama3.1", "prompt": "Hey! How's it going?", "stream": False,
                      "options": {"temperature": 0, "num_predict": 12}})
    cs = ClusterServer("tiny-llama", gpus=1, device="cuda", sd_seed=3, warmup=False, kv_pages=64)
    try:
        got = json.loads(cs.handle_json(req))
        m = cs.metrics()
    finally:
        cs.close()
    assert got["eval_count"] == 12 and m["live_replicas"] == 1

    import torch

    from p2p_llm_chat_go_amd.engine import Engine
    from p2p_llm_chat_go_amd.engine.server import EngineServer
    from p2p_llm_chat_go_amd.models.config import get_config
    from p2p_llm_chat_go_amd.models.reference import random_state_dict
    from p2p_llm_chat_go_amd.models.weights import EngineWeights

    cfg = get_config("tiny-llama")
    w = EngineWeights.from_state_dict(random_state_dict(cfg, seed=3), cfg, "cuda")
    srv = EngineServer(Engine(cfg, weights=w, device="cuda", kv_pages=64))
    try:
        ref = json.loads(srv.handle_json(req))
    finally:
        srv.close()
    assert torch.cuda.is_available()
    assert got["response"] == ref["response"]
