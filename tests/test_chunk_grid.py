"""The two chunk grids of csum_kernel (csrc/xcsum_kernels.hip, resolve<DW>
and the edge masks), restated in Python and checked exhaustively over frame
phase and length: every byte the kernel loads lies inside the frame's own
memory -- never before the Ethernet header, never past the 16-byte block
(aligned grid) or the dword (dword grid) holding the frame's last byte, so a
frame ending at the end of a mapping can not fault -- and the bytes kept
after masking are exactly the checksum span.  Host-only model test."""
import pytest


def grid(eth, length, family, dw):
    hdr, pre = (54, 32) if family == 6 else (34, 8)
    lo = eth + hdr - pre
    hi = eth + length
    if dw:
        e4 = (hi + 3) & ~3
        n = (e4 - lo + 15) >> 4
        base = e4 - 16 * n
        head, tail = lo - base, e4 - hi
        # kept: chunk 0 drops bytes [0, head); the last chunk's top `tail`
        # bytes of its last dword
        kept = set(range(base, base + 16 * n)) - set(range(base, base + head)) \
            - set(range(e4 - tail, e4))
    else:
        base = lo & ~15
        n = (hi - base + 15) >> 4
        head, tail = lo - base, 16 * n - (hi - base)
        kept = set(range(base, base + 16 * n)) - set(range(base, base + head)) \
            - set(range(base + 16 * n - tail, base + 16 * n))
    return base, n, head, tail, kept, lo, hi


@pytest.mark.parametrize("dw", [False, True])
@pytest.mark.parametrize("family", [4, 6])
def test_grid_reads_stay_inside_the_frame(dw, family):
    hdr = 54 if family == 6 else 34
    for eth in range(64, 80):                       # every 16-byte phase
        for length in list(range(hdr + 8, hdr + 200)) + [1514, 1534, 9042, 65535 + hdr]:
            base, n, head, tail, kept, lo, hi = grid(eth, length, family, dw)
            assert 0 <= head <= 15
            assert 0 <= tail <= (3 if dw else 15)
            assert base >= eth                       # nothing before the frame
            end = base + 16 * n
            limit = ((hi + 3) & ~3) if dw else (((hi - 1) | 15) + 1)
            assert end <= limit                      # nothing past hi's dword / block
            assert base % (4 if dw else 16) == 0     # dword / 16-byte aligned loads
            assert kept == set(range(lo, hi))        # exactly the span survives
            # a one-chunk frame gets both masks on the same chunk: disjoint
            if n == 1:
                assert head + tail <= 16
