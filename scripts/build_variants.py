"""Build A/B variants of libarctopk next to the product library (CPU; hipcc cross-compiles).

    python scripts/build_variants.py NAME:DEF1,DEF2 NAME2:DEF ...
-> allreducetopk_amd/lib/var/libarctopk_NAME.so (select with ARCTOPK_LIB, scripts/gpu_ab.sh)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import build as B  # noqa: E402


def one(spec):
    name, _, defs = spec.partition(":")
    defines = [d for d in defs.split(",") if d]
    out = os.path.join(B.LIBDIR, "var", f"libarctopk_{name}.so")
    B.build(out=out, defines=defines)
    return out


if __name__ == "__main__":
    B.build()
    with ThreadPoolExecutor(2) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)
