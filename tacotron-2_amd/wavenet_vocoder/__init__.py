"""Reference-compatible ``wavenet_vocoder`` package (code/wavenet_vocoder/) backed by libtt2.so."""
