"""Native byte-level BPE tokenizer (csrc/engine/bpe_tok.h) against the HF `tokenizers`
library: a Llama-3-style tokenizer.json (BPE trained here on chat text over the byte-level
alphabet, the Llama-3 Split pattern + ByteLevel pre-tokenizer, ignore_merges, the Llama-3
special tokens appended after the vocab as in the real file) must give the same prompt ids
and the same decoded text through the engine C ABI's probe as through Python's HFTokenizer,
on ASCII and non-ASCII chat text (with TOKENIZER_PATH set no request
needs the interpreter).  Parity is pinned to the installed `tokenizers`; code points whose
letter / number class changed across Unicode versions are "parity unpinned"."""
import json
import random

import pytest

from p2p_llm_chat_go_amd.engine.tokenizer import SAMPLE_MESSAGES, HFTokenizer, suggest_prompt
from tokutil import NON_ASCII, train_bpe_tokenizer as _train

tokenizers = pytest.importorskip("tokenizers")

def _texts():
    rng = random.Random(11)
    alpha = "abcXYZ019_ .,!?'\"-:;()\n\t\r  @#$%^&*[]{}<>/\\|`~+=éüßñ日本語Жж😀½²  "
    out = list(SAMPLE_MESSAGES) + [suggest_prompt(m) for m in SAMPLE_MESSAGES] + NON_ASCII
    out += ["", " ", "\n\n", "don't", "it's 6pm", "I'M HERE", "we'VE", "__init__", "..."]
    for _ in range(300):
        out.append("".join(rng.choice(alpha) for _ in range(rng.randrange(0, 48))))
    return out


@pytest.mark.parametrize("gpt2", [False, True], ids=["llama3", "gpt2"])
def test_native_bpe_ids_equal_tokenizers(probe, tmp_path, gpt2):
    tok = HFTokenizer(_train(tmp_path, gpt2=gpt2))
    spec = tok.native_spec()
    assert spec["kind"] == "bpe"
    for t in _texts():
        r = probe(spec, {"prompt": t})
        assert r["native"], repr(t)
        assert r["ids"] == tok.chat_ids(t), repr(t)
        r = probe(spec, {"prompt": t, "raw": True})
        assert r["native"] and r["ids"] == tok.encode(t, bos=True), repr(t)
    msgs = [{"role": "system", "content": "Sé breve."}, {"role": "user", "content": "Привет!"},
            {"role": "assistant", "content": "Hi 😀"}, {"role": "user", "content": "Lunch at noon?"}]
    for k in range(len(msgs) + 1):
        r = probe(spec, {"endpoint": "chat", "messages": msgs[:k]})
        assert r["native"] and r["ids"] == tok.chat_messages_ids(msgs[:k]), k


def test_native_bpe_decode_equals_tokenizers(probe, tmp_path):
    tok = HFTokenizer(_train(tmp_path))
    spec = tok.native_spec()
    n = tok.tok.get_vocab_size()
    rng = random.Random(7)
    lists = [tok.chat_ids(t) for t in _texts()[:80]]
    # random ids: byte tokens that split multi-byte characters (U+FFFD), specials, unknown ids
    lists += [[rng.randrange(0, n + 3) for _ in range(rng.randrange(0, 40))] for _ in range(200)]
    for ids in lists:
        assert probe(spec, {"prompt": ""}, ids)["text"] == tok.decode(ids), ids


def test_uncovered_tokenizer_json_falls_back_to_python(probe, tmp_path):
    tok = HFTokenizer(_train(tmp_path, normalizer="nfkc"))
    assert not probe(tok.native_spec(), {"prompt": "hello"})["native"]
    (tmp_path / "b").mkdir()
    spec = HFTokenizer(_train(tmp_path / "b")).native_spec()
    assert probe(spec, {"prompt": "hello"})["native"]


def test_explicit_nulls_take_the_python_path(probe, tmp_path):
    """Python renders an explicit null role / content as "None" and raises on a
    null prompt; only a missing key takes the default natively."""
    spec = HFTokenizer(_train(tmp_path)).native_spec()
    assert not probe(spec, {"endpoint": "chat", "messages": [{"role": None, "content": "hi"}]})["native"]
    assert not probe(spec, {"endpoint": "chat", "messages": [{"role": "user", "content": None}]})["native"]
    assert not probe(spec, {"prompt": None})["native"]
    assert not probe(spec, {"prompt": None, "raw": True})["native"]
    assert probe(spec, {"endpoint": "chat", "messages": [{"content": "hi"}]})["native"]
    assert probe(spec, {})["native"]
