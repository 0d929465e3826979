"""C2 and C4 (-m bsf and -m sf) on the full-size BASELINE stand-in genome: hg19 contig lengths,
i.i.d. ACGT with hg19-like N-gap runs (tools/synth.genome_ngaps, what bench.py measures).  As in
test_gpu_configs.py: a large batch on the GPU, a random sample plus every read that needed a search
tier >= 1 compared byte for byte with the oracle, whose index takes the GPU suffix arrays only after
the complete O(n) check of both."""
import os
import sys
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from test_gpu_configs import O, _batch_and_check, _say, _threads, synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hg19_full(request):
    import gwa
    t0 = time.time()
    codes, names, lengths = synth.genome_ngaps(synth.HG19_CONTIGS, config_id=1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    _say(request, "hg19 (N gaps) genome + GPU index in %.0fs" % (time.time() - t0))
    t0 = time.time()
    T = _threads()
    sa_f = gi.suffixArray(0)
    O.check_cyclic_sa_full(codes, sa_f, threads=T)
    sa_r = gi.suffixArray(1)
    O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=T)
    oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
    del sa_f, sa_r
    _say(request, "complete SA check + oracle index in %.0fs" % (time.time() - t0))
    yield codes, names, lengths, gi, oi
    gi.close()


@pytest.mark.timeout(900)
def test_c2_full_size_hg19_k2(hg19_full, request):
    """C2: 100 bp, 0-2 substitutions, -k 2, -m bsf: 2M reads, 200k random + every tier >= 1 read."""
    codes, names, lengths, gi, oi = hg19_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 2_000_000, 100, 2, config_id=2))
    _batch_and_check(request, gi, oi, strs, 100, 2.0, "bsf", 200_000)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("strategy", ["bsf", "sf"])
def test_c4_full_size_hg19_indels_k5(hg19_full, request, strategy):
    """C4: 150 bp, 0-5 edits with 1-bp indels, -k 5: 100k reads, 50k random + every tier >= 1 read."""
    codes, names, lengths, gi, oi = hg19_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 100_000, 150, 2, config_id=4, indels=True,
                                              max_edits=5))
    _batch_and_check(request, gi, oi, strs, 150, 5.0, strategy, 50_000)
