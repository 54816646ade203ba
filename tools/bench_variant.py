"""bench.py against a variant package tree (tools/build_variant.sh / build_rev.sh): the package
directory CPG_DEV_PKG goes first on sys.path, then bench.main() runs with this command line's
arguments.  Development A/B only — bench.py itself loads the in-tree build and nothing else.
usage: CPG_DEV_PKG=build/abl/pkg_<name> python tools/bench_variant.py --steps 400 ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv[0] = os.path.join(ROOT, "bench.py")
import bench  # noqa: E402  (puts ROOT first on sys.path; imports no package module yet)

if os.environ.get("CPG_DEV_PKG"):
    sys.path.insert(0, os.path.abspath(os.environ["CPG_DEV_PKG"]))
assert "cpgisland_amd" not in sys.modules
import inspect  # noqa: E402

from cpgisland_amd import hmm as _hmm  # noqa: E402  (the variant's)

if "chunk_len" not in inspect.signature(_hmm.Context.reserve).parameters:
    # an older revision's Context: reserve() sizes for every chunk length anyway
    _reserve = _hmm.Context.reserve
    _hmm.Context.reserve = lambda self, n, general=False, chunk_len=None: _reserve(self, n, general)

if __name__ == "__main__":
    bench.main()
