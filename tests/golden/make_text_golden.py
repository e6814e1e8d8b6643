"""Generate tests/golden/text_frontend.json (+ tests/golden/tiny_bpe.model) from the REFERENCE
text front-end and host helpers.  Run in the build container only:
``python tests/golden/make_text_golden.py``

Covers ``indextts/utils/front.py`` (TextNormalizer with an identity TN grammar plugged in --
WeTextProcessing is absent here --, TextTokenizer.tokenize / split_sentences / decode),
``indextts/utils/common.py`` (tokenize_by_CJK_char / de_tokenized_by_CJK_char) and
``IndexTTS.bucket_sentences`` / ``IndexTTS.pad_tokens_cat`` (``indextts/infer.py:188-262``, called on
an instance created without ``__init__``).  Shims: stub ``torchaudio`` / ``omegaconf`` modules
(imported but unused on these paths).  The SentencePiece model is trained here on a small synthetic
corpus (the real ``bpe.model`` is not available offline) and committed as fixture data.
"""
from __future__ import annotations

import importlib.machinery
import json
import warnings
import os
import random
import sys
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("ITTS_REFERENCE", "/root/reference")

import transformers  # noqa: E402,F401  (must precede the torchaudio stub)

for name in ("torchaudio", "omegaconf"):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    m.OmegaConf = None
    sys.modules.setdefault(name, m)
_mpu = types.ModuleType("transformers.utils.model_parallel_utils")  # removed in transformers 5.x
_mpu.assert_device_map = _mpu.get_device_map = lambda *a, **k: None
sys.modules["transformers.utils.model_parallel_utils"] = _mpu
sys.path.insert(0, REF)

from indextts.utils.common import de_tokenized_by_CJK_char, tokenize_by_CJK_char  # noqa: E402
from indextts.utils.front import TextNormalizer, TextTokenizer  # noqa: E402
from indextts.infer import IndexTTS  # noqa: E402

TEXTS = [
    "IndexTTS 正式发布1.0版本了，效果666",
    "晕XUAN4是一种GAN3觉",
    "晕 XUAN4 是 一 种 GAN3 觉",
    "我爱你！",
    "I love you!",
    "“我爱你”的英语是“I love you”",
    "受不liao3你了",
    "“衣裳”不读衣chang2，而是读衣shang5",
    "最zhong4要的是：不要chong2蹈覆辙",
    "不zuo1死就不会死",
    "See you at 8:00 AM",
    "Couting down 3, 2, 1, go!",
    "这酒...里...有毒...",
    "只有,,,才是最好的",
    "babala2是什么？",
    "用beta1测试",
    "have you ever been to beta2?",
    "where's the money?",
    "今天是个好日子 it's a good day",
    "约瑟夫·高登-莱维特（Joseph Gordon-Levitt is an American actor）",
    "电影1：“黑暗骑士”（演员：克里斯蒂安·贝尔、希斯·莱杰；导演：克里斯托弗·诺兰）；电影2：“盗梦空间”",
    "There is a vehicle arriving in dock number 7? Please stand clear. The doors are closing - mind the gap!",
    "hello@example.com",
    "嗯，呣……好吧。",
    "x",
    "",
    "ju4 que4 xue2 lü4",
    "He said: 'stop'. Then he left! Did he? Yes... he did.",
]

CORPUS_EXTRA = [
    "the quick brown fox jumps over the lazy dog", "mind the gap between the train and the platform",
    "我们今天去公园散步，天气非常好。", "他说这件事情很重要，必须马上处理！", "你知道吗？这个问题很难回答。",
    "please stand clear of the closing doors", "number seven dock arriving vehicle",
]


def train_bpe(path):
    import sentencepiece as spm
    lines = []
    for t in TEXTS + CORPUS_EXTRA:
        if t.strip():
            lines.append(tokenize_by_CJK_char(t))
    corpus = os.path.join(HERE, "_bpe_corpus.txt")
    with open(corpus, "w", encoding="utf-8") as f:
        for _ in range(20):
            f.write("\n".join(lines) + "\n")
    prefix = path[: -len(".model")]
    spm.SentencePieceTrainer.train(input=corpus, model_prefix=prefix, vocab_size=300, model_type="bpe",
                                   character_coverage=1.0, num_threads=1, bos_id=0, eos_id=1, unk_id=2, pad_id=-1,
                                   user_defined_symbols=["'", "▁'"], hard_vocab_limit=False)
    os.remove(corpus)
    os.remove(prefix + ".vocab")


class _Identity:
    def normalize(self, text):
        return text


def _split(fn, *a):
    """reference result, or the exception name (some inputs recurse without end in the reference:
    an over-long run holding both ',' and '-' alternates between the two re-splits)"""
    try:
        return fn(*a)
    except RecursionError:
        return "RecursionError"


def main():
    warnings.simplefilter("ignore")
    sys.setrecursionlimit(400)
    rng = random.Random(0)
    out = {}
    bpe = os.path.join(HERE, "tiny_bpe.model")
    train_bpe(bpe)
    norm = TextNormalizer()
    norm.zh_normalizer = norm.en_normalizer = _Identity()
    TextNormalizer.load = lambda self: None  # keep the identity grammar
    tok = TextTokenizer(bpe, norm)
    out["cjk"] = [[t, tokenize_by_CJK_char(t), tokenize_by_CJK_char(t, do_upper_case=False)] for t in TEXTS]
    out["de_cjk"] = [[s, de_tokenized_by_CJK_char(s), de_tokenized_by_CJK_char(s, do_lower_case=True)]
                     for s in [c[1] for c in out["cjk"]]]
    out["use_chinese"] = [[t, bool(norm.use_chinese(t))] for t in TEXTS]
    out["correct_pinyin"] = [[p, norm.correct_pinyin(p)] for p in
                             ["ju4", "que4", "xue2", "lü4", "xün1", "jian1", "zhong4", "JU3", "qun2", "xuan4"]]
    out["normalize"] = [[t, norm.normalize(t)] for t in TEXTS]
    rows = []
    for t in TEXTS:
        toks = tok.tokenize(t)
        ids = tok.encode(t)
        rows.append({"text": t, "tokens": toks, "ids": ids, "decode": tok.decode(ids),
                     "split": {str(m): _split(tok.split_sentences, toks, m) for m in (4, 8, 20, 120)}})
    out["tokenizer"] = rows
    # split_sentences_by_token on synthetic token streams
    alphabet = [".", "!", "?", "▁.", "▁?", "▁...", ",", "▁,", "-", "'", "▁'", "▁A", "B", "C", "▁D", "E", "F"]
    weights = [2, 1, 1, 2, 1, 1, 3, 3, 2, 2, 2, 8, 8, 8, 8, 8, 8]
    split_cases = []
    for i in range(300):
        n = rng.choice([0, 1, 2, 3, 5, 9, 17, 33, 64])
        seq = rng.choices(alphabet, weights=weights, k=n)
        mx = rng.choice([2, 3, 4, 6, 8, 16, 40])
        split_cases.append({"tokens": seq, "max": mx,
                            "out": _split(TextTokenizer.split_sentences_by_token, seq,
                                          TextTokenizer.punctuation_marks_tokens, mx)})
    out["split_by_token"] = split_cases
    # IndexTTS.bucket_sentences / pad_tokens_cat on an instance built without __init__
    tts = IndexTTS.__new__(IndexTTS)
    buckets = []
    for i in range(120):
        n = rng.choice([1, 2, 3, 4, 5, 7, 9, 13, 20])
        sents = [["x"] * rng.choice([0, 1, 2, 3, 5, 8, 12, 20, 33]) for _ in range(n)]
        bms = rng.choice([1, 2, 3, 4, 6])
        res = tts.bucket_sentences(sents, bucket_max_size=bms)
        buckets.append({"lens": [len(s) for s in sents], "bucket_max_size": bms,
                        "out": [[d["idx"] for d in b] for b in res]})
    out["bucket_sentences"] = buckets

    class _Cfg:
        class gpt:
            stop_text_token = 1
            start_text_token = 0

    pads = []
    for version in (1.5, None):
        tts.model_version = version
        tts.cfg = _Cfg
        for i in range(20):
            toks = [torch.randint(2, 100, (1, rng.randint(1, 15)), generator=torch.Generator().manual_seed(100 * i + j),
                                  dtype=torch.int32) for j in range(rng.randint(1, 5))]
            res = tts.pad_tokens_cat(toks)
            pads.append({"version": version, "in": [t[0].tolist() for t in toks], "out": res.tolist()})
    out["pad_tokens_cat"] = pads
    path = os.path.join(HERE, "text_frontend.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes;", bpe, os.path.getsize(bpe), "bytes")


if __name__ == "__main__":
    main()
