"""Text front-end of ``IndexTTS.infer``: normalisation, CJK pre-tokenisation, SentencePiece ids and
sentence splitting.  Host-side (pure Python); it feeds the GPU path token ids.

Restates the reference's ``indextts/utils/front.py`` (``TextNormalizer`` :11-229,
``TextTokenizer`` :232-429) and ``indextts/utils/common.py`` (``tokenize_by_CJK_char`` :29-52,
``de_tokenized_by_CJK_char`` :55-81).  The number/date verbalisation inside ``normalize`` is the
third-party WeTextProcessing (``tn.chinese`` / ``tn.english``, or ``wetext`` on macOS), which is
not in this image: ``TextNormalizer.load`` uses it when importable and otherwise installs an
identity normaliser (logged once) -- everything around it (pinyin-tone / name protection,
contraction rewrite, punctuation maps) is reproduced and pinned against the reference with an
identity normaliser plugged into both (tests/golden/text_frontend.json).
"""
from __future__ import annotations

import os
import re
import sys
import warnings
from typing import Dict, List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------------------------
# CJK pre-tokeniser (common.py:29-81)
# ---------------------------------------------------------------------------------------------
_CJK = re.compile(
    r"([\u1100-\u11ff\u2e80-\ua4cf\ua840-\uD7AF\uF900-\uFAFF\uFE30-\uFE4F\uFF65-\uFFDC\U00020000-\U0002FFFF])")


def tokenize_by_CJK_char(line: str, do_upper_case: bool = True) -> str:
    """Space-separate every CJK character; other runs are kept (upper-cased by default)."""
    parts = (w.strip() for w in _CJK.split(line.strip()))
    return " ".join(w.upper() if do_upper_case else w for w in parts if w)


_EN_RUN = re.compile(r"([A-Z]+(?:[\s-][A-Z-]+)*)", re.IGNORECASE)
_PLACEHOLDER = re.compile(r"^.*?(<sent_(\d+)>)")


def de_tokenized_by_CJK_char(line: str, do_lower_case: bool = False) -> str:
    """Inverse of :func:`tokenize_by_CJK_char`: drop the spaces but keep English phrases intact."""
    runs = _EN_RUN.findall(line)
    for i, r in enumerate(runs):
        line = line.replace(r, f"<sent_{i}>")
    out = []
    for w in line.split():
        m = _PLACEHOLDER.match(w)
        if m:
            w = w.replace(m.group(1), runs[int(m.group(2))])
            if do_lower_case:
                w = w.lower()
        out.append(w)
    return "".join(out)


# ---------------------------------------------------------------------------------------------
# normaliser (front.py:11-229)
# ---------------------------------------------------------------------------------------------
_PUNCT_MAP: Dict[str, str] = {
    "：": ",", "；": ",", ";": ",", "，": ",", "。": ".", "！": "!", "？": "?", "\n": " ", "·": "-", "、": ",",
    "...": "…", ",,,": "…", "，，，": "…", "……": "…", "“": "'", "”": "'", '"': "'", "‘": "'", "’": "'",
    "（": "'", "）": "'", "(": "'", ")": "'", "《": "'", "》": "'", "【": "'", "】": "'", "[": "'", "]": "'",
    "—": "-", "～": "-", "~": "-", "「": "'", "」": "'", ":": ",",
}
_ZH_PUNCT_MAP: Dict[str, str] = {"$": ".", **_PUNCT_MAP}


def _replacer(table: Dict[str, str]):
    # alternation in insertion order (first listed alternative wins at a position, like the reference)
    pat = re.compile("|".join(re.escape(k) for k in table))
    return lambda s: pat.sub(lambda m: table[m.group()], s)


class _Identity:
    def normalize(self, text: str) -> str:
        return text


class TextNormalizer:
    PINYIN_TONE_PATTERN = (r"(?<![a-z])((?:[bpmfdtnlgkhjqxzcsryw]|[zcs]h)?(?:[aeiouüv]|[ae]i|u[aio]|ao|ou|i[aue]|"
                           r"[uüv]e|[uvü]ang?|uai|[aeiuv]n|[aeio]ng|ia[no]|i[ao]ng)|ng|er)([1-5])")
    NAME_PATTERN = r"[\u4e00-\u9fff]+(?:[-·—][\u4e00-\u9fff]+){1,2}"
    ENGLISH_CONTRACTION_PATTERN = r"(what|where|who|which|how|t?here|it|s?he|that|this)'s"

    def __init__(self):
        self.zh_normalizer = None
        self.en_normalizer = None
        self.char_rep_map = dict(_PUNCT_MAP)
        self.zh_char_rep_map = dict(_ZH_PUNCT_MAP)
        self._sub = _replacer(self.char_rep_map)
        self._zh_sub = _replacer(self.zh_char_rep_map)

    # -- WeTextProcessing (third party) --
    def load(self):
        if self.zh_normalizer is not None and self.en_normalizer is not None:
            return
        try:
            import platform
            if platform.system() == "Darwin":
                from wetext import Normalizer
                self.zh_normalizer = Normalizer(remove_erhua=False, lang="zh", operator="tn")
                self.en_normalizer = Normalizer(lang="en", operator="tn")
            else:
                from tn.chinese.normalizer import Normalizer as NormalizerZh
                from tn.english.normalizer import Normalizer as NormalizerEn
                cache_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tagger_cache")
                os.makedirs(cache_dir, exist_ok=True)
                self.zh_normalizer = NormalizerZh(cache_dir=cache_dir, remove_interjections=False, remove_erhua=False,
                                                  overwrite_cache=False)
                self.en_normalizer = NormalizerEn(overwrite_cache=False)
        except ImportError:
            print(">> WeTextProcessing is not installed: numbers/dates are not verbalised "
                  "(identity text normaliser)", file=sys.stderr)
            self.zh_normalizer = self.en_normalizer = _Identity()

    @staticmethod
    def match_email(s: str) -> bool:
        return re.match(r"^[a-zA-Z0-9]+@[a-zA-Z0-9]+\.[a-zA-Z]+$", s) is not None

    def use_chinese(self, s: str) -> bool:
        if re.search(r"[\u4e00-\u9fff]", s) or not re.search(r"[a-zA-Z]", s) or self.match_email(s):
            return True
        return bool(re.search(self.PINYIN_TONE_PATTERN, s, re.IGNORECASE))

    # placeholders <tag_a>, <tag_b>, ... protect spans from the TN grammar
    @staticmethod
    def _protect(text: str, pattern: str, tag: str) -> Tuple[str, Optional[List[str]]]:
        found = re.findall(re.compile(pattern, re.IGNORECASE), text)
        if not found:
            return text, None
        spans = list(set("".join(f) if isinstance(f, tuple) else f for f in found))
        for i, sp in enumerate(spans):
            text = text.replace(sp, f"<{tag}_{chr(ord('a') + i)}>")
        return text, spans

    @staticmethod
    def _restore(text: str, spans: Optional[List[str]], tag: str, fix=None) -> str:
        for i, sp in enumerate(spans or ()):
            text = text.replace(f"<{tag}_{chr(ord('a') + i)}>", fix(sp) if fix else sp)
        return text

    def save_pinyin_tones(self, text: str):
        return self._protect(text, self.PINYIN_TONE_PATTERN, "pinyin")

    def restore_pinyin_tones(self, text: str, spans):
        return self._restore(text, spans, "pinyin", self.correct_pinyin)

    def save_names(self, text: str):
        return self._protect(text, self.NAME_PATTERN, "n")

    def restore_names(self, text: str, spans):
        return self._restore(text, spans, "n")

    @staticmethod
    def correct_pinyin(pinyin: str) -> str:
        """j/q/x + u/ü finals are written with v (ju -> JV); result upper-cased."""
        if pinyin[0] not in "jqxJQX":
            return pinyin
        return re.sub(r"([jqx])[uü](n|e|an)*(\d)", r"\g<1>v\g<2>\g<3>", pinyin, flags=re.IGNORECASE).upper()

    def normalize(self, text: str) -> str:
        text = text.replace("嗯", "恩").replace("呣", "母")
        if not self.zh_normalizer or not self.en_normalizer:
            print("Error, text normalizer is not initialized !!!")
            return ""
        zh = self.use_chinese(text)  # decided before the contraction rewrite (front.py:118-119)
        text = re.sub(self.ENGLISH_CONTRACTION_PATTERN, r"\1 is", text, flags=re.IGNORECASE)
        if zh:
            work, pinyin = self.save_pinyin_tones(text.rstrip())
            work, names = self.save_names(work)
            try:
                work = self.zh_normalizer.normalize(work)
            except Exception:  # the reference logs and returns "" on a TN failure
                import traceback
                print(traceback.format_exc())
                work = ""
            work = self.restore_pinyin_tones(self.restore_names(work, names), pinyin)
            return self._zh_sub(work)
        try:
            work = self.en_normalizer.normalize(text)
        except Exception:
            import traceback
            print(traceback.format_exc())
            work = text
        return self._sub(work)


# ---------------------------------------------------------------------------------------------
# tokenizer + sentence splitting (front.py:232-429)
# ---------------------------------------------------------------------------------------------
def split_sentences_by_token(tokens: Sequence[str], split_tokens: Sequence[str],
                             max_tokens_per_sentence: int) -> List[List[str]]:
    """Cut after a split token (once a sentence has > 2 tokens); an over-long run is re-split at
    commas, then at hyphens, then every ``max_tokens_per_sentence`` tokens; finally neighbours whose
    joint length fits are merged.  Reproduces the reference exactly, including that a quote
    following a split token is appended to the finished sentence *and* starts the next one
    (front.py:363-368 bumps a for-loop variable, which has no effect)."""
    if not tokens:
        return []
    out: List[List[str]] = []
    cur: List[str] = []
    for i, tok in enumerate(tokens):
        cur.append(tok)
        if len(cur) <= max_tokens_per_sentence:
            if tok in split_tokens and len(cur) > 2:
                done = cur + ([tokens[i + 1]] if i + 1 < len(tokens) and tokens[i + 1] in ("'", "▁'") else [])
                out.append(done)
                cur = []
            continue
        # over-long: cur holds max + 1 tokens
        has_comma_split = "," in split_tokens or "▁," in split_tokens
        if not has_comma_split and ("," in cur or "▁," in cur):
            out.extend(split_sentences_by_token(cur, [",", "▁,"], max_tokens_per_sentence))
        elif "-" not in split_tokens and "-" in cur:
            out.extend(split_sentences_by_token(cur, ["-"], max_tokens_per_sentence))
        else:
            out.extend(cur[j: j + max_tokens_per_sentence] for j in range(0, len(cur), max_tokens_per_sentence))
            warnings.warn(f"The tokens length of sentence exceeds limit: {max_tokens_per_sentence}, "
                          f"Tokens in sentence: {cur}.Maybe unexpected behavior", RuntimeWarning)
        cur = []
    if cur:
        out.append(cur)
    merged: List[List[str]] = []
    for s in out:
        if not s:
            continue
        if merged and len(merged[-1]) + len(s) <= max_tokens_per_sentence:
            merged[-1] = merged[-1] + s
        else:
            merged.append(s)
    return merged


class TextTokenizer:
    punctuation_marks_tokens = [".", "!", "?", "▁.", "▁?", "▁..."]

    def __init__(self, vocab_file: str, normalizer: Optional[TextNormalizer] = None):
        if vocab_file is None:
            raise ValueError("vocab_file is None")
        if not os.path.exists(vocab_file):
            raise ValueError(f"vocab_file {vocab_file} does not exist")
        from sentencepiece import SentencePieceProcessor
        self.vocab_file = vocab_file
        self.normalizer = normalizer
        if normalizer:
            normalizer.load()
        self.sp_model = SentencePieceProcessor(model_file=vocab_file)
        self.pre_tokenizers = [tokenize_by_CJK_char]

    # special ids of the IndexTTS text vocabulary
    unk_token, pad_token, bos_token, eos_token = "<unk>", None, "<s>", "</s>"
    pad_token_id, bos_token_id, eos_token_id = -1, 0, 1

    @property
    def vocab_size(self) -> int:
        return self.sp_model.GetPieceSize()

    @property
    def unk_token_id(self) -> int:
        return self.sp_model.unk_id()

    @property
    def special_tokens_map(self):
        return {"unk_token": self.unk_token, "pad_token": self.pad_token, "bos_token": self.bos_token,
                "eos_token": self.eos_token}

    def get_vocab(self):
        return {self.convert_ids_to_tokens(i): i for i in range(self.vocab_size)}

    def convert_ids_to_tokens(self, ids):
        return self.sp_model.IdToPiece(ids)

    def convert_tokens_to_ids(self, tokens) -> List[int]:
        if isinstance(tokens, str):
            tokens = [tokens]
        return [self.sp_model.PieceToId(t) for t in tokens]

    def _prepare(self, text: str) -> str:
        if self.normalizer:
            text = self.normalizer.normalize(text)
        for pre in self.pre_tokenizers:
            text = pre(text)
        return text

    def encode(self, text: str, **kwargs):
        out_type = kwargs.pop("out_type", int)
        if len(text) == 0:
            return []
        if len(text.strip()) == 1:  # a single character skips normalisation (front.py:320-321)
            return self.sp_model.Encode(text, out_type=out_type, **kwargs)
        return self.sp_model.Encode(self._prepare(text), out_type=out_type, **kwargs)

    def tokenize(self, text: str) -> List[str]:
        return self.encode(text, out_type=str)

    def batch_encode(self, texts: List[str], **kwargs):
        return self.sp_model.Encode([self._prepare(t) for t in texts], out_type=kwargs.pop("out_type", int), **kwargs)

    def decode(self, ids, do_lower_case: bool = False, **kwargs):
        if isinstance(ids, int):
            ids = [ids]
        text = self.sp_model.Decode(ids, out_type=kwargs.pop("out_type", str), **kwargs)
        return de_tokenized_by_CJK_char(text, do_lower_case=do_lower_case)

    split_sentences_by_token = staticmethod(split_sentences_by_token)

    def split_sentences(self, tokenized: List[str], max_tokens_per_sentence: int = 120) -> List[List[str]]:
        return split_sentences_by_token(tokenized, self.punctuation_marks_tokens, max_tokens_per_sentence)
