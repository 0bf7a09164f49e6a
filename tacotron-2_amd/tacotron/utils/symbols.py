"""Symbol set of code/tacotron/utils/symbols.py:9-17: pad '_', EOS '~', 66 symbols in total.

The ARPAbet extension is commented out in the fork (symbols.py:14,17), so ``{...}`` spans in
``text_to_sequence`` map to nothing, exactly as in the reference.
"""
_pad = '_'
_eos = '~'
_characters = 'ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz!\'\"(),-.:;? '

symbols = [_pad, _eos] + list(_characters)
