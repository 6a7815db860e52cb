"""Write the 'large' (or PHMM_KIND) phmm job as a .in file (PairHMMUnitTest.cpp's input) for bin/phmm.
    python tools/phmm_write_in.py /tmp/large.in
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import gen  # noqa: E402

gen.write_phmm_file(sys.argv[1], gen.phmm_dataset(os.environ.get("PHMM_KIND", "large"),
                                                  int(os.environ.get("PHMM_BATCHES", "64")), seed=1))
