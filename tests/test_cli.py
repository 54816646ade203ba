"""CPU checks of the command-line driver (cpgisland_amd.cli, CpGIslandFinder.main :346-357):
argument handling and the Java int arithmetic of the reference's logged count (:107, :147).
The end-to-end run is tests/test_gpu_cli.py."""
from cpgisland_amd import cli


def test_usage_without_six_arguments():
    assert cli.main(["a", "b"]) == 2


def test_java_int_wrap():
    assert cli._java_int(5) == 5
    assert cli._java_int((1 << 31) + 3) == -(1 << 31) + 3
    assert cli._java_int(1 << 32) == 0
