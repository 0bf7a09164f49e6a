"""Runs named test functions of tests/test_train.py in order, in this (fresh) process.

Used by tests/test_gpu_memcheck.py: the library reads TT2_POISON_ALLOC / TT2_REDZONE once per
process, and an order-dependent failure needs a process whose allocation history is exactly the
listed tests.  Usage: python tests/_memcheck_run.py name[:arg,arg] ...
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tacotron-2_amd"), os.path.join(HERE, ".."), HERE]

import test_train  # noqa: E402


def _arg(s):
    if s in ("True", "False"):
        return s == "True"
    return int(s)


for spec in sys.argv[1:]:
    name, _, args = spec.partition(":")
    fn = getattr(test_train, name)
    fn(*[_arg(a) for a in args.split(",") if a])
    print("ok", spec, flush=True)
print("__MEMCHECK_OK__", flush=True)
