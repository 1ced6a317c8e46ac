"""Debug: golden kurtosis case on the GPU vs emulations (leaf path)."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import conftest as C
orc = C.entry.load_oracle()
pkg = C.entry.load_package()
eng = pkg.engine
g = C.Golden()
c = g.cases("kurtosis")[0]
a = g.input(c["input"]); win = c["win"]
x = eng.fb_from_numpy(a, device="cuda:0")
print(eng.kurtosis_plan(x, win))
got = eng.fb_to_numpy(eng.kurtosis(x, win)).reshape(-1, order="F")
want = orc.kurtosis(a, win).reshape(-1, order="F")
w = orc.np_window(a, win); nc, ni, nt = w.shape
rows = w.reshape((nc * ni, nt), order="F").astype(np.float64)
m = orc.mean_f32(a, win).reshape(-1, order="F").astype(np.float64)
d = rows - m[:, None]
emu = (d ** 4).mean(1) / ((d ** 2).mean(1)) ** 2 - 3
fin = np.isfinite(want)
r = np.abs(got - want) / (C.KURT_LEAF_TOL * np.abs(want + 3))
r[~fin] = 0
for i in np.argsort(r)[-6:]:
    print(i, r[i], got[i], want[i], emu[i], got[i] - emu[i], rows[i].max(), rows[i, 0], m[i])
# the unaligned (two-pass, recipe) path on the same data
a2 = np.asfortranarray(np.concatenate([a[:1], a], axis=0))
x2 = eng.fb_from_numpy(a2, device="cuda:0")
w2 = [1, a.shape[0], 1, 0, a.shape[1], 1, 0, a.shape[2], 1]
print(eng.kurtosis_plan(x2, w2))
tp = eng.fb_to_numpy(eng.kurtosis(x2, w2)).reshape(-1, order="F")
print("twopass max rel", np.nanmax(np.abs(tp - want)[fin] / np.abs(want[fin] + 3)))
