"""The plugin's film hand-over: a live imageFilm_t gives its
filterTable and filterw; yk_film_filter_from_table names the filter by
comparing the table with the four libyk builds (imagefilm.cc:119-165) and
refuses anything else, so a film libyk cannot reproduce fails loudly instead of
rendering with the wrong filter. The tables here come from the oracle's own
restatement of the film constructor."""
import ctypes as C

import numpy as np
import pytest

from core_amd import _abi as A
from oracle.oracle import film_table

FILTERS = [A.YK_FILTER_BOX, A.YK_FILTER_MITCHELL, A.YK_FILTER_GAUSS, A.YK_FILTER_LANCZOS]


def _params(filt, pw):
    p = A.yk_render_params()
    A.lib().yk_render_params_default(C.byref(p))
    p.filter = filt
    p.aa_pixelwidth = pw
    return p


def _identify(table, fw):
    q = A.yk_render_params()
    A.lib().yk_render_params_default(C.byref(q))
    rc = A.lib().yk_film_filter_from_table(table.ctypes.data_as(A.fp), fw, C.byref(q))
    return rc, q


@pytest.mark.parametrize("pw", [1.0, 1.5, 2.2, 4.0])
@pytest.mark.parametrize("filt", FILTERS)
def test_filter_identified_from_the_film_table(filt, pw):
    table, fw = film_table(_params(filt, pw))
    rc, q = _identify(table, fw)
    assert rc == A.YK_OK, A.lib().yk_last_error()
    assert q.filter == filt and q.filter_width == np.float32(fw)


def test_unknown_table_or_width_refused():
    table, fw = film_table(_params(A.YK_FILTER_MITCHELL, 1.5))
    bad = table.copy()
    bad[17] = np.nextafter(bad[17], np.float32(2))  # one ulp off: not a table libyk builds
    assert _identify(bad, fw)[0] == A.YK_ERR_UNSUPPORTED
    assert _identify(table, 4.5)[0] == A.YK_ERR_UNSUPPORTED  # > MAX_FILTER_SIZE / 2
    assert _identify(table, 0.4)[0] == A.YK_ERR_UNSUPPORTED


def test_filter_width_overrides_pixelwidth_in_the_oracle():
    """filter_width carries the film's filterw as is; aa_pixelwidth is then
    ignored (both the oracle and libyk's make_film)."""
    p = _params(A.YK_FILTER_GAUSS, 1.5)
    p.filter_width = 1.25
    _, fw = film_table(p)
    assert fw == np.float32(1.25)
