"""Character ids for Tacotron (the behaviour of code/tacotron/utils/text.py:1-74).

Input text is cut into plain runs and curly-brace ARPAbet spans with the reference's span grammar
(text.py:30-38: shortest prefix, first ``{...}``, remainder; ``.`` stops at a newline, so the
remainder after a newline is dropped exactly as there).  Plain runs go through the named cleaners,
ARPAbet words become ``@``-prefixed symbols -- which the fork's symbol set does not contain
(symbols.py:14,17), so they contribute no ids.  Symbols outside the table, the pad ``_`` and the
EOS ``~`` are skipped (text.py:73-74), and one EOS id is appended (text.py:40-41).
"""
import functools
import re

from . import cleaners
from .symbols import symbols

_PAD, _EOS = '_', '~'
_ID = {s: i for i, s in enumerate(symbols)}
_SYMBOL = dict(enumerate(symbols))
_EMITTED = frozenset(s for s in symbols if s not in (_PAD, _EOS))
_SPAN = re.compile(r'(.*?)\{(.+?)\}(.*)')


def _segments(text):
    """Yield (is_arpabet, piece) in text order."""
    while text:
        m = _SPAN.match(text)
        if m is None:
            yield False, text
            return
        prefix, phones, text = m.groups()
        yield False, prefix
        yield True, phones


def _cleaned(text, cleaner_names):
    fns = []
    for name in cleaner_names:
        fn = getattr(cleaners, name, None)
        if fn is None:
            raise Exception('Unknown cleaner: %s' % name)
        fns.append(fn)
    return functools.reduce(lambda acc, fn: fn(acc), fns, text)


def text_to_sequence(text, cleaner_names):
    """Ids of ``text`` after ``cleaner_names``, EOS-terminated."""
    ids = []
    for is_arpabet, piece in _segments(text):
        syms = ['@' + p for p in piece.split()] if is_arpabet else _cleaned(piece, cleaner_names)
        ids.extend(_ID[s] for s in syms if s in _EMITTED)
    ids.append(_ID[_EOS])
    return ids


def sequence_to_text(sequence):
    """Inverse mapping; ARPAbet symbols render as ``{...}`` with adjacent spans space-joined."""
    pieces = []
    for i in sequence:
        s = _SYMBOL.get(i)
        if s is None:
            continue
        pieces.append('{%s}' % s[1:] if len(s) > 1 and s.startswith('@') else s)
    return ''.join(pieces).replace('}{', ' ')
