"""the npz hand-off files of the DDP -> SCP -> DDP pipeline, in the
reference's layouts (demos/*.ipynb np.savez calls; src/whole_body_control.py:41-44;
src/centroidal_model.py:174)."""
import numpy as np

from cmpc import npz_io


def test_warm_start_round_trip_and_truncation(tmp_path):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(3, 31, 9))
    paths = npz_io.save_warm_start(str(tmp_path / npz_io.WARM_START), X)
    assert len(paths) == 3 and all(p.endswith('.npz') for p in paths)
    # the reference's reader: np.load(...)['X'].T is (9, N+1)
    assert np.load(paths[1])['X'].T.shape == (9, 31)
    np.testing.assert_array_equal(npz_io.load_warm_start(paths, 30), X)
    np.testing.assert_array_equal(npz_io.load_warm_start(paths[0], 20)[0], X[0, :21])


def test_to_whole_body_layout(tmp_path):
    N = 20
    rng = np.random.default_rng(1)
    res = [dict(state=[rng.normal(size=(9, N + 1))], control=[rng.normal(size=(12, N))], gains=[], covs=[]),
           False, dict(state=[], control=[], gains=[], covs=[])]
    out = npz_io.save_to_whole_body(str(tmp_path / npz_io.TO_WHOLE_BODY), res)
    assert out[1] is None and out[2] is None
    X, U = npz_io.load_tracking(out[0])
    assert X.shape == (9, N + 1) and U.shape == (12, N)
    np.testing.assert_array_equal(X, res[0]['state'][-1])
    single = npz_io.save_to_whole_body(str(tmp_path / 'single.npz'), res[0])
    assert single == [str(tmp_path / 'single.npz')]


def test_interpolated_files(tmp_path):
    d = dict(X=np.ones((9, 200)), U=np.zeros((12, 190)))
    p = npz_io.save_interpolated(str(tmp_path / 'scp_sol_interpol_nom.npz'), d)[0]
    f = np.load(p)
    assert f['X'].shape == (9, 200) and f['U'].shape == (12, 190)
