"""Import-compatible alias of the reference module ``indextts/utils/front.py``
(``from indextts.utils.front import TextNormalizer, TextTokenizer``); see :mod:`indextts.utils.text`."""
from .text import TextNormalizer, TextTokenizer, de_tokenized_by_CJK_char, tokenize_by_CJK_char  # noqa: F401
