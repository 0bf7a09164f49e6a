"""Text frontend (tacotron/utils: symbols, cleaners, numbers, text) — CPU.

The reference's text.py/cleaners.py/numbers.py need unidecode + inflect (absent), so nothing can
be generated from the reference here: the expectations below restate the behaviour those modules
document (symbols.py:9-17, text.py:14-74, cleaners.py:80-87, numbers.py:43-69).  Parity unpinned
for the inflect-worded numbers beyond these cases.
"""
import numpy as np
import pytest

from tacotron.utils import cleaners
from tacotron.utils.numbers import _number_to_words, normalize_numbers
from tacotron.utils.symbols import symbols
from tacotron.utils.text import sequence_to_text, text_to_sequence


def test_symbol_table_matches_reference_size():
    assert len(symbols) == 66  # hparams/tacotron.py embedding table rows
    assert symbols[0] == '_' and symbols[1] == '~' and symbols[-1] == ' '


def test_eos_appended_and_round_trip():
    seq = text_to_sequence("Hello, world!", ["basic_cleaners"])
    assert seq[-1] == 1
    assert sequence_to_text(seq) == "hello, world!~"
    assert all(2 <= i < 66 for i in seq[:-1])


def test_pad_and_eos_symbols_dropped_and_unknown_skipped():
    seq = text_to_sequence("a_b~c#", ["basic_cleaners"])
    assert sequence_to_text(seq) == "abc~"


def test_curly_braces_arpabet_maps_to_nothing_in_fork_symbols():
    # the fork comments the ARPAbet symbols out (symbols.py:14,17): braces contribute no ids
    seq = text_to_sequence("Turn left on {HH AW1 S S T AH0 N} Street.", ["english_cleaners"])
    assert sequence_to_text(seq) == "Turn left on  Street.~"


@pytest.mark.parametrize("num,words", [
    (0, "zero"), (7, "seven"), (13, "thirteen"), (40, "forty"), (99, "ninety-nine"),
    (100, "one hundred"), (101, "one hundred and one"), (999, "nine hundred and ninety-nine"),
    (1000, "one thousand"), (3456, "three thousand, four hundred and fifty-six"),
    (1000000, "one million"), (2000005, "two million, five"),
])
def test_cardinals(num, words):
    assert _number_to_words(num) == words


@pytest.mark.parametrize("s,words", [
    ("1st", "first"), ("2nd", "second"), ("3rd", "third"), ("12th", "twelfth"),
    ("20th", "twentieth"), ("21st", "twenty-first"), ("100th", "one hundredth"),
    ("101st", "one hundred and first"), ("55th", "fifty-fifth"),
])
def test_ordinals(s, words):
    assert _number_to_words(s) == words


@pytest.mark.parametrize("text,out", [
    ("1984", "nineteen eighty-four"), ("1905", "nineteen oh five"), ("2000", "two thousand"),
    ("2007", "two thousand seven"), ("1100", "eleven hundred"), ("2019", "twenty nineteen"),
    ("3456", "three thousand, four hundred fifty-six"), ("1,000,000", "one million"),
    ("$3.50", "three dollars, fifty cents"), ("$1", "one dollar"), ("$0.01", "one cent"),
    ("$0", "zero dollars"), ("2.5", "two point five"), ("21st", "twenty-first"),
])
def test_normalize_numbers(text, out):
    assert cleaners.collapse_whitespace(normalize_numbers(text)) == out


def test_english_cleaners_pipeline():
    t = cleaners.english_cleaners("Dr. Müller paid  $3.50 on   the 2nd of May 1984.")
    # no lowercasing in the fork (cleaners.py:83 commented out), abbreviations expanded after
    # numbers, whitespace collapsed, umlaut transliterated
    assert t == "doctor Muller paid three dollars, fifty cents on the second of May nineteen eighty-four."


def test_transliteration_cleaners():
    assert cleaners.transliteration_cleaners("Ça  Va? Straße") == "ca va? strasse"


def test_pound_sign_is_transliterated_before_number_expansion():
    # english_cleaners runs convert_to_ascii first, so '£' (unidecode: 'PS') never reaches the
    # pounds rule of normalize_numbers (cleaners.py:81-84)
    assert cleaners.english_cleaners("£20") == "PStwenty"


def test_unknown_cleaner_raises():
    with pytest.raises(Exception):
        text_to_sequence("x", ["no_such_cleaner"])
