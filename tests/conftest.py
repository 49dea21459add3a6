"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on any host (oracle vs golden fixtures, host logic, the
C ABI's exports).  `-m gpu` runs the parity tests through librsac.so on an
MI355X and must not be skipped silently: they fail if no device is present.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "code-reproduction-ransac_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built librsac.so")
