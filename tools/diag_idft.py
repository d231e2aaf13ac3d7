import sys, numpy as np
sys.path.insert(0, '.')
import openair4g_amd as oai
oai.init()
z = np.load('tests/golden/idft_ref.npz')
for key in z.files:
    if key.startswith('x_2048'):
        _, size, vi, scale = key.split('_')
        y = oai.idft(z[key], int(scale)); ref = z[f'y_{size}_{vi}_{scale}']
        d = np.nonzero(y != ref)[0]
        print(key, len(d), d[:40] // 2, (y[d[:10]].astype(int) - ref[d[:10]]))
rng = np.random.default_rng(1)
x = rng.integers(-300, 300, 4096).astype(np.int16)
y1 = oai.idft(x, 1); y2 = oai.idft(x, 1)
print("repeat equal", np.array_equal(y1, y2))
x = np.zeros(4096, np.int16); x[0] = 1000
print("impulse", oai.idft(x, 0)[:8])
