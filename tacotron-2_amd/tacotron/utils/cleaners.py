"""Cleaners of code/tacotron/utils/cleaners.py:1-90 (names and pipelines unchanged).

``convert_to_ascii`` replaces ``unidecode`` (absent here) with Unicode NFKD decomposition,
combining marks dropped, a small table for letters NFKD leaves alone (ß, æ, ø, ł, đ, þ, œ and
typographic punctuation), and anything still non-ASCII removed.  That matches unidecode on
Latin-script text (the reference's English corpora); other scripts are not transliterated.
Note the fork's ``english_cleaners`` does NOT lowercase (cleaners.py:83 is commented out).
"""
import re
import unicodedata

from .numbers import normalize_numbers

_whitespace_re = re.compile(r'\s+')

_abbreviations = [(re.compile('\\b%s\\.' % x[0], re.IGNORECASE), x[1]) for x in [
    ('mrs', 'misess'), ('mr', 'mister'), ('dr', 'doctor'), ('st', 'saint'), ('co', 'company'),
    ('jr', 'junior'), ('maj', 'major'), ('gen', 'general'), ('drs', 'doctors'),
    ('rev', 'reverend'), ('lt', 'lieutenant'), ('hon', 'honorable'), ('sgt', 'sergeant'),
    ('capt', 'captain'), ('esq', 'esquire'), ('ltd', 'limited'), ('col', 'colonel'),
    ('ft', 'fort'),
]]

_ASCII_EXTRA = {
    'ß': 'ss', 'æ': 'ae', 'Æ': 'AE', 'ø': 'o', 'Ø': 'O', 'ł': 'l', 'Ł': 'L', 'đ': 'd', 'Đ': 'D',
    'þ': 'th', 'Þ': 'Th', 'œ': 'oe', 'Œ': 'OE', 'ð': 'd', 'Ð': 'D', 'ı': 'i',
    '£': 'PS', '€': 'EUR', '‘': "'", '’': "'", '‚': ',', '“': '"', '”': '"', '„': ',,', '–': '-', '—': '--',
    '…': '...', '«': '<<', '»': '>>', ' ': ' ',
}


def expand_abbreviations(text):
    for regex, replacement in _abbreviations:
        text = re.sub(regex, replacement, text)
    return text


def expand_numbers(text):
    return normalize_numbers(text)


def lowercase(text):
    return text.lower()


def collapse_whitespace(text):
    return re.sub(_whitespace_re, ' ', text)


def convert_to_ascii(text):
    out = []
    for ch in text:
        if ord(ch) < 128:
            out.append(ch)
            continue
        if ch in _ASCII_EXTRA:
            out.append(_ASCII_EXTRA[ch])
            continue
        d = unicodedata.normalize('NFKD', ch)
        out.append(''.join(c for c in d if ord(c) < 128 and not unicodedata.combining(c)))
    return ''.join(out)


def basic_cleaners(text):
    text = lowercase(text)
    text = collapse_whitespace(text)
    return text


def transliteration_cleaners(text):
    text = convert_to_ascii(text)
    text = lowercase(text)
    text = collapse_whitespace(text)
    return text


def english_cleaners(text):
    """cleaners.py:80-87 (no lowercase in the fork)."""
    text = convert_to_ascii(text)
    text = expand_numbers(text)
    text = expand_abbreviations(text)
    text = collapse_whitespace(text)
    return text
