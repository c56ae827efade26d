"""The kernel-source fingerprint a committed profile records (bench.kernel_build_id)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build_id():
    import bench
    return bench.kernel_build_id()
