"""Reference-compatible ``tacotron`` package (code/tacotron/) backed by libtt2.so."""
