"""Tokenizers and the suggest-reply prompt.

* ``HFTokenizer`` loads a real ``tokenizer.json`` (Llama-3 tiktoken-BPE or
  Mixtral SentencePiece exported to HF format) through the ``tokenizers``
  package when a file is supplied (``TOKENIZER_PATH`` or a checkpoint dir).
* ``SyntheticTokenizer`` is the offline default (no tokenizer files on the
  box): a deterministic word-level tokenizer whose token counts track BPE on
  English chat text (one token per word / punctuation mark), which is all the
  benchmark depends on.  Ids are stable hashes into the model vocabulary.
  Decoding is a pure function of the id, identical in every process (DP replicas,
  TP ranks, the node): ids of a fixed built-in vocabulary (common chat words, the
  co-pilot template, the sample messages) decode to their word, every other id to a
  deterministic pronounceable pseudo-word -- never to whatever this process happened
  to encode before.

``suggest_prompt`` reproduces the reference co-pilot template verbatim
(`web/streamlit_app.py:93`) and ``chat_ids`` wraps it the way Ollama's
llama3.1 template does (one user turn, assistant header open).
"""
from __future__ import annotations

import os
import re
import zlib

SUGGEST_TEMPLATE = ("You are a helpful assistant. Draft a concise, friendly reply to the following "
                    "message:\n\n{prompt}\n\nReply:")

LLAMA3_SPECIAL = {
    "<|begin_of_text|>": 128000, "<|end_of_text|>": 128001, "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007, "<|eom_id|>": 128008, "<|eot_id|>": 128009,
}


def suggest_prompt(message: str) -> str:
    return SUGGEST_TEMPLATE.format(prompt=message)


def _render_messages(tok, messages: list, special) -> list:
    """Ollama ``/api/chat`` messages -> prompt ids, per-message roles kept.

    llama3.x (Ollama's llama3.1 template): ``<|begin_of_text|>`` then, per message,
    ``<|start_header_id|>{role}<|end_header_id|>\n\n{content}<|eot_id|>``, then an open
    assistant header.  [INST] models (Mixtral): a system message is prepended to the
    first user turn; assistant turns close with ``</s>``."""
    msgs = [m for m in messages or [] if isinstance(m, dict)]
    if tok.llama3:
        ids = [tok.bos_id]
        for m in msgs:
            ids += [special("<|start_header_id|>")] + tok.encode(str(m.get("role", "user")))
            ids += [special("<|end_header_id|>")] + tok.encode("\n\n" + str(m.get("content", "")))
            ids += [special("<|eot_id|>")]
        return ids + [special("<|start_header_id|>")] + tok.encode("assistant") + [
            special("<|end_header_id|>")] + tok.encode("\n\n")
    ids = [tok.bos_id]
    system = "\n\n".join(str(m.get("content", "")) for m in msgs if m.get("role") == "system")
    for m in msgs:
        role, content = m.get("role", "user"), str(m.get("content", ""))
        if role == "system":
            continue
        if role == "assistant":
            ids += tok.encode(" " + content) + list(tok.eos_ids[:1])
            continue
        if system:
            content, system = system + "\n\n" + content, ""
        ids += tok.encode("[INST] " + content + " [/INST]")
    return ids


# Built-in vocabulary of the synthetic tokenizer: decoding these words is exact.
_COMMON = (
    "a about after again all also am an and any are around as at back be been before being "
    "best better but by call can could day did do does done don't down each even every find "
    "first for from get give go going good got great had has have he hear hello help her here "
    "hey hi him his hope how i if in into is it it's just know last let like look lot love make "
    "many maybe me meet more morning most much my need new next nice night no not now of off "
    "ok okay on one only or other our out over please plan really right said same see send she "
    "should so some soon sorry sounds still sure take talk team tell than thank thanks that "
    "the their them then there these they thing think this time to today tomorrow too two up "
    "us very want was way we week well were what when where which while who why will with "
    "work would yeah yes yet you your happy glad free later tonight weekend lunch dinner "
    "coffee meeting project call message reply friend great awesome cool definitely absolutely "
    "let's see you soon")


class SyntheticTokenizer:
    _pat = re.compile(r"\s*\w+|\s*[^\w\s]|\s+")
    _tables: dict = {}  # (lo, hi) -> {id: piece}, shared by every instance of a vocab range

    def __init__(self, vocab: int = 128256, n_special: int = 256, bos_id=None, eos_ids=None,
                 llama3: bool | None = None):
        self.vocab = vocab
        self.llama3 = vocab >= 128256 if llama3 is None else llama3
        self.hi = vocab - n_special if not self.llama3 else 128000
        self.lo = 3
        self.bos_id = bos_id if bos_id is not None else (128000 if self.llama3 else 1)
        self.eos_ids = tuple(eos_ids) if eos_ids else ((128009, 128001) if self.llama3 else (2,))

    def _id(self, piece: str) -> int:
        h = zlib.crc32(piece.encode("utf-8"))
        return self.lo + h % (self.hi - self.lo)

    def _table(self) -> dict:
        key = (self.lo, self.hi)
        t = SyntheticTokenizer._tables.get(key)
        if t is None:
            corpus = [_COMMON, SUGGEST_TEMPLATE, "user assistant system"] + list(SAMPLE_MESSAGES)
            pieces = set()
            for text in corpus:
                for m in self._pat.finditer(text):
                    w = m.group(0)
                    for v in (w.strip(), w.strip().capitalize()):
                        pieces.update((v, " " + v, "\n" + v, "\n\n" + v))
                    pieces.add(w)
            pieces.update(("\n\n", "\n", " "))
            t = {}
            for w in sorted(p for p in pieces if p):  # sorted: collisions resolve the same way
                t.setdefault(self._id(w), w)
            SyntheticTokenizer._tables[key] = t
        return t

    @staticmethod
    def _pseudo(i: int) -> str:
        """Deterministic pronounceable word for an id outside the built-in vocabulary."""
        cons, vows = "bdfgklmnprstvz", "aeiou"
        out = []
        n = int(i)
        while True:
            out.append(cons[n % len(cons)] + vows[(n // len(cons)) % len(vows)])
            n //= len(cons) * len(vows)
            if n == 0:
                break
        return " " + "".join(out)

    def encode(self, text: str, bos: bool = False) -> list:
        ids = [self.bos_id] if bos else []
        ids += [self._id(m.group(0)) for m in self._pat.finditer(text) if m.group(0)]
        return ids

    def decode(self, ids) -> str:
        out = []
        inv = {v: k for k, v in LLAMA3_SPECIAL.items()} if self.llama3 else {}
        table = self._table()
        for i in ids:
            i = int(i)
            if i in inv or i == self.bos_id or i in self.eos_ids:
                continue
            w = table.get(i)
            out.append(w if w is not None else self._pseudo(i))
        return "".join(out).strip()

    def chat_ids(self, user_text: str) -> list:
        if self.llama3:
            S = LLAMA3_SPECIAL
            ids = [S["<|begin_of_text|>"], S["<|start_header_id|>"]] + self.encode("user") + [
                S["<|end_header_id|>"]] + self.encode("\n\n" + user_text) + [S["<|eot_id|>"],
                                                                           S["<|start_header_id|>"]]
            return ids + self.encode("assistant") + [S["<|end_header_id|>"]] + self.encode("\n\n")
        return [self.bos_id] + self.encode("[INST] " + user_text + " [/INST]")

    def chat_messages_ids(self, messages: list) -> list:
        return _render_messages(self, messages, LLAMA3_SPECIAL.__getitem__)

    def native_spec(self) -> dict:
        """What the engine C ABI needs to encode / decode natively (csrc/engine/
        native_tok.h): the hash range, the special ids and the built-in decode table; ids
        outside the table decode to ``_pseudo`` words, which the native side recomputes."""
        return {"kind": "synthetic", "llama3": bool(self.llama3), "lo": self.lo, "hi": self.hi,
                "bos": int(self.bos_id), "eos": [int(e) for e in self.eos_ids],
                "special": dict(LLAMA3_SPECIAL) if self.llama3 else {},
                "pieces": [[int(i), w] for i, w in sorted(self._table().items())]}


class HFTokenizer:
    def __init__(self, path: str, eos_ids=None):
        from tokenizers import Tokenizer

        if os.path.isdir(path):
            path = os.path.join(path, "tokenizer.json")
        self.path = os.path.abspath(path)
        self.tok = Tokenizer.from_file(path)
        self.vocab = self.tok.get_vocab_size()
        self.llama3 = self.tok.token_to_id("<|begin_of_text|>") is not None
        if self.llama3:
            self.bos_id = self.tok.token_to_id("<|begin_of_text|>")
        else:
            self.bos_id = self.tok.token_to_id("<s>") or 1
        self.eos_ids = tuple(eos_ids) if eos_ids else tuple(
            i for i in (self.tok.token_to_id("<|eot_id|>"), self.tok.token_to_id("<|end_of_text|>"),
                        self.tok.token_to_id("</s>")) if i is not None)

    def encode(self, text: str, bos: bool = False) -> list:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] if bos else []) + ids

    def decode(self, ids) -> str:
        return self.tok.decode([int(i) for i in ids], skip_special_tokens=True).strip()

    def chat_ids(self, user_text: str) -> list:
        if self.llama3:
            t = self.tok.token_to_id
            return ([self.bos_id, t("<|start_header_id|>")] + self.encode("user")
                    + [t("<|end_header_id|>")] + self.encode("\n\n" + user_text)
                    + [t("<|eot_id|>"), t("<|start_header_id|>")] + self.encode("assistant")
                    + [t("<|end_header_id|>")] + self.encode("\n\n"))
        return [self.bos_id] + self.encode("[INST] " + user_text + " [/INST]")

    def chat_messages_ids(self, messages: list) -> list:
        return _render_messages(self, messages, self.tok.token_to_id)

    def native_spec(self) -> dict:
        """The engine C ABI reads the same tokenizer.json natively (csrc/engine/bpe_tok.h:
        byte-level BPE with the Llama-3 or GPT-2 pre-tokenizer, as Llama-3's); a file with
        parts it does not implement (a SentencePiece-style model such as Mixtral's, a
        normalizer, ...) is refused there and every request asks Python to encode / decode."""
        special = {k: self.tok.token_to_id(k) for k in LLAMA3_SPECIAL}
        return {"kind": "bpe", "path": self.path, "llama3": bool(self.llama3),
                "bos": int(self.bos_id), "eos": [int(e) for e in self.eos_ids],
                "special": {k: int(v) for k, v in special.items() if v is not None}}


def get_tokenizer(cfg=None, path: str | None = None):
    path = path or os.environ.get("TOKENIZER_PATH")
    if path and os.path.exists(path):
        return HFTokenizer(path, eos_ids=getattr(cfg, "eos_ids", None))
    if cfg is None:
        return SyntheticTokenizer()
    return SyntheticTokenizer(vocab=cfg.vocab, bos_id=cfg.bos_id, eos_ids=cfg.eos_ids,
                              llama3=cfg.vocab >= 128256)


# Synthetic incoming chat messages (the screenshot's kind of traffic).
SAMPLE_MESSAGES = [
    "Hey! How's it going?",
    "Are we still on for lunch tomorrow at noon? I can book a table near the office.",
    "Thanks for sending the slides yesterday, they looked great. Any chance you could add the Q3 numbers?",
    "I just landed in Berlin, the flight was delayed by two hours. Can we move our call to 6pm?",
    "Did you see the game last night? That last-minute goal was unbelievable!",
    "Quick question: do you know where the spare keys for the storage room are?",
    "Happy birthday!! Hope you have an amazing day and a great year ahead.",
    "My laptop keeps freezing when I open the project, have you seen this before?",
]
