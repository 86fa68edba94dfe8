"""Multi-locus step host logic (BASELINE config 5): the 734-region table
parser, per-locus path templates, round-robin assignment of loci to ranks."""
import pytest

from grid_amd.utils.hi_inference import _locus_path, read_loci_file
from tests.loci_cohort import LOCI_TABLE


def test_read_734_region_table():
    loci = read_loci_file(LOCI_TABLE)
    assert len(loci) == 734
    assert loci[0] == {"chrom": "1", "start": 939399, "end": 939508, "gene": "SAMD11", "index": 0}
    # gene names repeat, regions do not: the default {locus} name is unique
    assert len({lc["gene"] for lc in loci}) < 734
    names = {str(_locus_path("{locus}", lc)) for lc in loci}
    assert len(names) == 734
    assert all(lc["start"] <= lc["end"] for lc in loci)


def test_loci_table_variants(tmp_path):
    p = tmp_path / "l.txt"
    p.write_text("chrom start end\nchr6 100 200\n\nchrX 5 9\n")
    loci = read_loci_file(p)
    assert [(lc["chrom"], lc["start"], lc["end"], lc["gene"]) for lc in loci] == \
        [("chr6", 100, 200, "chr6_100_200"), ("chrX", 5, 9, "chrX_5_9")]
    p.write_text("CHR\tGENE\n1\tA\n")
    with pytest.raises(ValueError):
        read_loci_file(p)
    p.write_text("CHR\tSTART\tEND\n1\tx\t5\n")
    with pytest.raises(ValueError):
        read_loci_file(p)


def test_round_robin_covers_every_locus_once():
    loci = read_loci_file(LOCI_TABLE)
    for world in (1, 2, 3, 8):
        got = sorted(lc["index"] for r in range(world) for lc in loci if lc["index"] % world == r)
        assert got == list(range(734))
