"""Build an A/B variant of libtreeinfer.so with extra compile flags into
kfserving_amd/lib/variants/NAME/ (git-ignored; it travels to the GPU box with
the tree), for scripts/ab_variant.sh:

    python scripts/build_variant.py NAME -DTI_T8_MASK=1 [-D...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import __graft_entry__ as g
    name, flags = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "kfserving_amd", "lib", "variants", name, "libtreeinfer.so")
    print(g.build_library(verbose=True, extra_flags=flags, lib=out))
