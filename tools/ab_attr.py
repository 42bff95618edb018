"""A/B of one PackedNet plan attribute on the bench (no environment knobs in the product):
    python tools/ab_attr.py fuse_pool2=0 -- --config K2 --steps 10 --warmup 2
sets the attribute on every PackedNet right after construction, then runs bench.main() with
the arguments after `--`."""
import os
import sys

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
sys.path.insert(0, os.path.join(os.path.dirname(here),
                                "federated-learning-for-privacy-preserving-image-classification_amd"))


def main():
    cut = sys.argv.index("--")
    sets = {}
    for kv in sys.argv[1:cut]:
        k, v = kv.split("=")
        sets[k] = bool(int(v))
    from fedhip import net
    init = net.PackedNet.__init__

    def patched(self, *a, **kw):
        init(self, *a, **kw)
        for k, v in sets.items():
            if not hasattr(self, k):
                raise AttributeError(f"PackedNet has no plan attribute {k}")
            setattr(self, k, v)

    net.PackedNet.__init__ = patched
    sys.argv = [sys.argv[0]] + sys.argv[cut + 1:]
    import bench
    bench.main()


if __name__ == "__main__":
    main()
