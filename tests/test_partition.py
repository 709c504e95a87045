"""Row partition planner (reference: rows/size, remainder dropped, kernel.cu:117)."""
import pytest

from mpi_cuda_imagemanipulation_amd import parallel


@pytest.mark.parametrize("H", [1, 2, 7, 8, 9, 100, 16384, 16385])
@pytest.mark.parametrize("N", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("R", [1, 2, 15])
def test_uneven_cover_exactly_once(H, N, R):
    stripes, active = parallel.plan_rows(H, N, R)
    assert len(stripes) == N
    covered = []
    for r, (row0, rows) in enumerate(stripes):
        if r < active:
            assert rows >= min(R, H)
            covered.extend(range(row0, row0 + rows))
        else:
            assert rows == 0
    assert covered == list(range(H))
    sizes = [rows for _, rows in stripes[:active]]
    assert max(sizes) - min(sizes) <= 1


def test_legacy_drops_remainder():
    stripes, active = parallel.plan_rows(10, 4, 1, True)
    assert [s[1] for s in stripes] == [2, 2, 2, 2]
    assert [s[0] for s in stripes] == [0, 2, 4, 6]


def test_too_many_ranks_shrinks_active():
    stripes, active = parallel.plan_rows(5, 8, 2)
    assert active == 2 and sum(s[1] for s in stripes) == 5
