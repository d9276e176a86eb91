"""bench.py with free_gpu() keeping torch's cached HBM blocks (gc only, no
empty_cache) -- placement probe for the extras that follow a large free.
    python tools/keep_cache_ab.py [bench.py args]"""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402

bench.free_gpu = lambda: gc.collect()
bench.main(sys.argv[1:])
