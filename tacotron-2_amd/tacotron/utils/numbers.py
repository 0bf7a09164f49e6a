"""Number normalisation of code/tacotron/utils/numbers.py:1-69 without ``inflect``.

The regex pipeline (commas, pounds, dollars, decimals, ordinals, cardinals; numbers.py:6-11,
62-69) and the year rules of ``_expand_number`` (:47-59) are the reference's.  The words come
from ``_number_to_words`` below, a restatement of ``inflect.engine().number_to_words`` for
non-negative integers: groups of three digits joined by ", ", "<h> hundred <andword> <tens>"
inside a group, hyphenated tens ("twenty-one"), ``group=2`` pair reading with ``zero`` for a
leading-zero pair ("nineteen oh five"), and ordinals ("twenty-first").  The cleaners collapse
the whitespace afterwards (cleaners.py:80-87), so inflect's double space around an empty
``andword`` disappears the same way.  Parity unpinned: inflect is absent and the reference has
no tests for this module.
"""
import re

_comma_number_re = re.compile(r'([0-9][0-9\,]+[0-9])')
_decimal_number_re = re.compile(r'([0-9]+\.[0-9]+)')
_pounds_re = re.compile(r'£([0-9\,]*[0-9]+)')
_dollars_re = re.compile(r'\$([0-9\.\,]*[0-9]+)')
_ordinal_re = re.compile(r'[0-9]+(st|nd|rd|th)')
_number_re = re.compile(r'[0-9]+')

_UNITS = ['', 'one', 'two', 'three', 'four', 'five', 'six', 'seven', 'eight', 'nine']
_TEENS = ['ten', 'eleven', 'twelve', 'thirteen', 'fourteen', 'fifteen', 'sixteen',
          'seventeen', 'eighteen', 'nineteen']
_TENS = ['', '', 'twenty', 'thirty', 'forty', 'fifty', 'sixty', 'seventy', 'eighty', 'ninety']
_MILLS = ['', ' thousand', ' million', ' billion', ' trillion', ' quadrillion', ' quintillion',
          ' sextillion', ' septillion', ' octillion', ' nonillion', ' decillion']
_ORD_EXC = {'one': 'first', 'two': 'second', 'three': 'third', 'five': 'fifth', 'eight': 'eighth',
            'nine': 'ninth', 'twelve': 'twelfth'}


def _tens(t, u):
    if t == 1:
        return _TEENS[u]
    if t:
        return _TENS[t] + ('-' + _UNITS[u] if u else '')
    return _UNITS[u]


def _group3(h, t, u, andword):
    """One three-digit group: '<h> hundred <andword> <tens>' (empty for 000)."""
    if h:
        mid = ' {} '.format(andword) if (t or u) else ''
        return '{} hundred{}{}'.format(_UNITS[h], mid, _tens(t, u))
    return _tens(t, u)


def _cardinal(num, andword):
    if num == 0:
        return 'zero'
    digits = str(num)
    groups = []
    while digits:
        groups.append(digits[-3:])
        digits = digits[:-3]
    words = []
    for mindex in range(len(groups) - 1, -1, -1):
        g = groups[mindex].rjust(3, '0')
        w = _group3(int(g[0]), int(g[1]), int(g[2]), andword)
        if w:
            words.append(w + _MILLS[mindex])
    return ', '.join(words)


def _pairs(num, zero):
    """group=2 reading: digit pairs from the left, '<zero> <unit>' for a '0d' pair, the last
    odd digit on its own."""
    s = str(num)
    out = []
    while len(s) >= 2:
        t, u = int(s[0]), int(s[1])
        if t == 0:
            out.append('{} {}'.format(zero, _UNITS[u]) if u else '{} {}'.format(zero, zero))
        else:
            out.append(_tens(t, u))
        s = s[2:]
    if s:
        out.append(_UNITS[int(s)] if s != '0' else zero)
    return ', '.join(out)


def _ordinalize(words):
    head, sep, last = words.rpartition(' ')
    pre, dash, lw = last.rpartition('-')
    if lw in _ORD_EXC:
        lw = _ORD_EXC[lw]
    elif lw.endswith('y'):
        lw = lw[:-1] + 'ieth'
    else:
        lw = lw + 'th'
    return head + sep + pre + dash + lw


def _number_to_words(num, andword='and', zero='zero', group=0):
    """inflect.engine().number_to_words for int or '<digits>(st|nd|rd|th)' strings."""
    ordinal = False
    if isinstance(num, str):
        m = re.match(r'^([0-9]+)(st|nd|rd|th)$', num)
        if m:
            ordinal = True
            num = int(m.group(1))
        else:
            num = int(num)
    words = _pairs(num, zero) if group == 2 else _cardinal(num, andword)
    return _ordinalize(words) if ordinal else words


def _plural(n, unit):
    return '%s %s' % (n, unit if n == 1 else unit + 's')


def _dollars(m):
    """numbers.py:22-40: '$1.50' -> '1 dollar, 50 cents'; more than one '.' is left as digits."""
    amount = m.group(1)
    whole, _, frac = amount.partition('.')
    if '.' in frac:
        return amount + ' dollars'
    d = int(whole) if whole else 0
    c = int(frac) if frac else 0
    said = [_plural(v, u) for v, u in ((d, 'dollar'), (c, 'cent')) if v]
    return ', '.join(said) if said else 'zero dollars'


def _cardinal_or_year(m):
    """numbers.py:47-59: integers in (1000, 3000) are read as years (2000 'two thousand', 2001-2009
    'two thousand <n>', whole hundreds '<nn> hundred', otherwise digit pairs with 'oh')."""
    n = int(m.group(0))
    if not 1000 < n < 3000:
        return _number_to_words(n, andword='')
    if n == 2000:
        return 'two thousand'
    if n < 2010 and n > 2000:
        return 'two thousand ' + _number_to_words(n % 100)
    if n % 100 == 0:
        return _number_to_words(n // 100) + ' hundred'
    return _number_to_words(n, andword='', zero='oh', group=2).replace(', ', ' ')


# numbers.py:62-69, applied in this order
_RULES = (
    (_comma_number_re, lambda m: m.group(1).replace(',', '')),
    (_pounds_re, lambda m: m.group(1) + ' pounds'),
    (_dollars_re, _dollars),
    (_decimal_number_re, lambda m: m.group(1).replace('.', ' point ')),
    (_ordinal_re, lambda m: _number_to_words(m.group(0))),
    (_number_re, _cardinal_or_year),
)


def normalize_numbers(text):
    """Spell out the numbers of ``text`` (numbers.py:62-69)."""
    for pattern, repl in _RULES:
        text = pattern.sub(repl, text)
    return text
