"""LDS image of k_gram8's 16x16x32 ring (LAY 4, grid_amd/csrc/knn.hip g8q_run),
checked on the host: the DMA pieces fill exactly the image the fragment reads
expect, and every ds_read_b128 lane group of a fragment read hits 16
distinct 16-B bank slots (conflict-free).  Lane groups of ds_read_b128 on
gfx950 (MI355X guide, LDS table): {0-3,12-15,20-27}, {4-11,16-19,28-31} and
the same +32."""

G = [0, 2, 3, 1]                                  # g8q_swz: (0x78 >> 2b) & 3


def swz(rb):
    return (0x78 >> (2 * (rb & 3))) & 3


LANE_GROUPS = [
    [*range(0, 4), *range(12, 16), *range(20, 28)],
    [*range(4, 12), *range(16, 20), *range(28, 32)],
]
LANE_GROUPS += [[x + 32 for x in g] for g in LANE_GROUPS]


def test_swizzle_table():
    assert [swz(b) for b in range(4)] == G


def test_dma_piece_fills_the_image_the_reads_expect():
    # piece = 16 rows x 64 B; lane i lands at LDS byte 16 i and loads row i >> 2,
    # logical chunk (i & 3) ^ g((i >> 4) & 3) of that row
    image = {}
    for i in range(64):
        row, j = i >> 2, (i & 3) ^ swz((i >> 4) & 3)
        image[16 * i] = (row, j)
    # fragment read: lane l wants row l & 15, logical chunk l >> 4, at
    # (l & 15) * 64 + ((l >> 4) ^ g((l >> 2) & 3)) * 16
    for l in range(64):
        addr = (l & 15) * 64 + (((l >> 4) ^ swz((l >> 2) & 3)) << 4)
        assert image[addr] == (l & 15, l >> 4), l


def test_fragment_reads_are_conflict_free():
    for base in (0, 1024, 4096, 16384):              # fragment / half / slot offsets are multiples of 1 KiB
        for grp in LANE_GROUPS:
            slots = set()
            for l in grp:
                addr = base + (l & 15) * 64 + (((l >> 4) ^ swz((l >> 2) & 3)) << 4)
                slots.add((addr // 16) % 16)         # 64 banks x 4 B = 16 slots of 16 B
            assert len(slots) == 16, (base, grp, sorted(slots))


def test_the_plain_row_swizzle_would_conflict():
    # the LAY 3 image's g = identity gives 2-way conflicts for these reads
    bad = 0
    for grp in LANE_GROUPS:
        slots = {((l & 15) * 64 + (((l >> 4) ^ ((l >> 2) & 3)) << 4)) // 16 % 16 for l in grp}
        bad += len(slots) < 16
    assert bad > 0
