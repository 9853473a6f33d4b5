"""A Llama-3-style byte-level BPE tokenizer.json built in-test with the `tokenizers` library
(no tokenizer files ship with the repo or the boxes): BPE trained on chat text over the
byte-level alphabet, the Llama-3 Split pattern + ByteLevel pre-tokenizer, ignore_merges,
and the Llama-3 special tokens appended after the vocab as in the real file."""
import tokenizers

from p2p_llm_chat_go_amd.engine.tokenizer import LLAMA3_SPECIAL, SAMPLE_MESSAGES, suggest_prompt

L3_PAT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
          r"|\s*[\r\n]+|\s+(?!\S)|\s+")

NON_ASCII = ["café au lait", "naïve résumé", "日本語のテキストです。", "Привет, как дела? Всё хорошо!",
             "emoji 😀👍🏽 fine", "Ünïcödé ÄÖÜ ß", "Ελληνικά κείμενα", "عربى نص", "한국어 문장",
             "non breaking spaces", "line sep", "x　y", "١٢٣ ٤٥٦ digits",
             "Ⅻ roman ½ fraction ²", "zero​width", "tab\tand\r\ncrlf \n\n end", "'ſ 'S 'LL 'Re",
             "mixed ASCII and 中文 together 123456789", "<|eot_id|> inside <|start_header_id|>text",
             "trailing spaces   ", "   leading", "a  b   c    d", "!!!???...", "(hello) [world] {x}"]


def train_bpe_tokenizer(tmp_path, pat=L3_PAT, gpt2=False, vocab=1500, normalizer=None):
    from tokenizers import Regex, Tokenizer, decoders, models, normalizers, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE(ignore_merges=not gpt2))
    if gpt2:
        tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    else:
        tok.pre_tokenizer = pre_tokenizers.Sequence([
            pre_tokenizers.Split(Regex(pat), behavior="isolated", invert=False),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    if normalizer:
        tok.normalizer = normalizers.NFKC()
    tok.decoder = decoders.ByteLevel()
    corpus = list(SAMPLE_MESSAGES) + [suggest_prompt(m) for m in SAMPLE_MESSAGES] + NON_ASCII
    tr = tokenizers.trainers.BpeTrainer(vocab_size=vocab, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                        show_progress=False)
    tok.train_from_iterator(corpus * 20, tr)
    tok.add_special_tokens(list(LLAMA3_SPECIAL))  # ids after the vocab, like Llama-3's 128000+
    path = tmp_path / "tokenizer.json"
    tok.save(str(path))
    return str(path)
