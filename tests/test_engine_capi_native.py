"""The engine C ABI's native request path (csrc/engine/engine_capi.cc, native_tok.h): the
prompt ids it builds from an Ollama request and the text it decodes must equal the Python
tokenizer's (engine/tokenizer.py) -- the C ABI serves requests without the interpreter
only if the two agree bit for bit.  Non-ASCII text must report "not native" (the request
then takes Python's tokenisation).  The reference sends the same prompt to Ollama
(`web/streamlit_app.py:91-95`); this is the in-process replacement's front end."""
import random

import pytest

from p2p_llm_chat_go_amd.engine.tokenizer import SAMPLE_MESSAGES, get_tokenizer, suggest_prompt
from p2p_llm_chat_go_amd.models import TINY_LLAMA
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B


def _texts():
    rng = random.Random(3)
    alphabet = "abcXYZ019_ .,!?'\"-:;()\n\t\r  @#$%^&*[]{}<>/\\|`~+="
    out = list(SAMPLE_MESSAGES) + [suggest_prompt(m) for m in SAMPLE_MESSAGES]
    out += ["", " ", "\n\n", "  leading", "trailing  ", "a\n\nb", "x  \n  y", "[INST] hi [/INST]",
            "don't", "it's 6pm", "__init__", "tabs\there", "..."]
    for _ in range(200):
        out.append("".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 40))))
    return out


@pytest.mark.parametrize("cfg", [TINY_LLAMA, LLAMA31_8B], ids=["tiny", "llama3"])
def test_native_prompt_ids_equal_python(probe, cfg):
    tok = get_tokenizer(cfg)
    spec = tok.native_spec()
    for t in _texts():
        r = probe(spec, {"prompt": t})
        assert r["native"] and r["ids"] == tok.chat_ids(t), repr(t)
        r = probe(spec, {"prompt": t, "raw": True})
        assert r["native"] and r["ids"] == tok.encode(t, bos=True), repr(t)
    msgs = [{"role": "system", "content": "Be brief."}, {"role": "user", "content": "Hey there!"},
            {"role": "assistant", "content": "Hi, what's up?"},
            {"role": "user", "content": "Lunch at noon?"}, {"role": "system", "content": ""}]
    for k in range(len(msgs) + 1):
        req = {"endpoint": "chat", "messages": msgs[:k]}
        r = probe(spec, req)
        assert r["native"] and r["ids"] == tok.chat_messages_ids(msgs[:k]), k


@pytest.mark.parametrize("cfg", [TINY_LLAMA, LLAMA31_8B], ids=["tiny", "llama3"])
def test_native_decode_equals_python(probe, cfg):
    tok = get_tokenizer(cfg)
    spec = tok.native_spec()
    rng = random.Random(5)
    lists = [tok.chat_ids(m) for m in SAMPLE_MESSAGES]
    lists += [[rng.randrange(0, cfg.vocab) for _ in range(rng.randrange(0, 50))] for _ in range(100)]
    lists.append(list(tok.eos_ids) + [tok.bos_id])
    for ids in lists:
        assert probe(spec, {"prompt": ""}, ids)["text"] == tok.decode(ids), ids


def test_non_ascii_and_odd_requests_fall_back_to_python(probe):
    spec = get_tokenizer(LLAMA31_8B).native_spec()
    assert not probe(spec, {"prompt": "café"})["native"]
    assert not probe(spec, {"prompt": "emoji \U0001F600"})["native"]
    assert not probe(spec, {"prompt": 42})["native"]
    assert not probe(spec, {"endpoint": "chat", "messages": [{"role": "user", "content": 3}]})["native"]
    assert not probe({"kind": "hf"}, {"prompt": "hello"})["native"]
    assert not probe(spec, {"endpoint": "chat", "messages": [{"role": None, "content": "x"}]})["native"]
