"""TEST INFRASTRUCTURE ONLY — CPU restatement (numpy) of the mwhitehill/Tacotron-2 inference path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / the timed CPU baseline.  The product path (``tacotron-2_amd``)
never imports it and has no CPU fallback.

Parity status: **parity unpinned**.  The reference is TensorFlow 1.x graph code with no tests, no
golden vectors and no trained Tacotron/WaveNet checkpoints; TensorFlow is not
installed here, so the reference cannot be run to produce outputs.  This restatement follows the
cited reference lines and the documented TF 1.x op semantics and is itself the
source of the committed golden fixtures under ``tests/golden/``.
"""
