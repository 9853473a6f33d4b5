"""Layouts the GEMM kernels rely on (CPU): fragment-major activations (ops.gemm.pack_frag)
and weights (tile_weight) follow the v_mfma_f32_16x16x32_bf16 operand layout."""
import torch

from p2p_llm_chat_go_amd.ops import gemm as G


def test_pack_frag_layout():
    torch.manual_seed(0)
    M, K = 37, 256
    x = torch.randn(M, K).to(torch.bfloat16)
    xp = G.pack_frag(x)
    assert xp.shape == (48, K)
    flat = xp.reshape(-1, 8)  # 16-byte chunks in (m-tile, k-step, lane) order
    S = K // 32
    for mt in range(3):
        for s in (0, S - 1):
            for lane in (0, 15, 16, 63):
                row, k = 16 * mt + (lane & 15), 32 * s + 8 * (lane >> 4)
                got = flat[(mt * S + s) * 64 + lane]
                want = x[row, k:k + 8] if row < M else torch.zeros(8, dtype=x.dtype)
                assert torch.equal(got, want), (mt, s, lane)


def test_tile_weight_roundtrip():
    w = torch.randn(64, 128).to(torch.bfloat16)
    assert torch.equal(G.untile_weight(G.tile_weight(w)), w)
