"""CPU restatement of the filter-feature branch's filters (test infrastructure).

Only tests/ import this.  It restates, in numpy, the rule
cluster_tools_amd/fastfilters.py implements on the GPU for the filters that
``vu.apply_filter`` (utils/volume_utils.py:80-94) looks up by name:
vigra-style Gaussian / Gaussian-derivative kernels (initGaussian /
initGaussianDerivative, radius int(3 sigma + 0.5 order + 0.5) [UPSTREAM,
unverified]) applied separably with mirror borders (numpy 'reflect' = vigra
BORDER_TREATMENT_REFLECT), and the per-voxel eigenvalues of the Hessian /
structure tensor with numpy.linalg.eigvalsh, descending.  fastfilters and
vigra are not in the image: parity against them is unpinned; this module pins
the GPU kernels to the stated rule.
"""
import numpy as np


def taps(sigma, order=0):
    """Correlation taps of the order-`order` Gaussian kernel."""
    if sigma <= 0:
        return np.ones(1)
    r = int(3.0 * sigma + 0.5 * order + 0.5)
    x = np.arange(-r, r + 1, dtype=np.float64)
    g = np.exp(-x * x / (2.0 * sigma * sigma))
    if order == 0:
        return g / g.sum()
    if order == 1:
        t = x / sigma ** 2 * g
        return t / np.sum(t * x)
    t = (x * x / sigma ** 4 - 1.0 / sigma ** 2) * g
    t = t - t.mean()
    return t / np.sum(t * x * x / 2.0)


def correlate_axis(a, axis, t):
    """out[p] = sum_k t[k] a[reflect(p + k - R)] along `axis` (float64)."""
    a = np.asarray(a, dtype=np.float64)
    r = t.size // 2
    if r == 0:
        return a * t[0]
    pad = [(0, 0)] * a.ndim
    pad[axis] = (r, r)
    ap = np.pad(a, pad, mode='reflect')
    out = np.zeros_like(a)
    n = a.shape[axis]
    for k in range(t.size):
        sl = [slice(None)] * a.ndim
        sl[axis] = slice(k, k + n)
        out += t[k] * ap[tuple(sl)]
    return out


def separable(a, sigmas, orders):
    out = np.asarray(a, dtype=np.float64)
    for ax, (s, o) in enumerate(zip(sigmas, orders)):
        out = correlate_axis(out, ax, taps(s, o))
    return out


def _sig(sigma, nd):
    return list(sigma) if isinstance(sigma, (list, tuple)) else [float(sigma)] * nd


def gaussianSmoothing(a, sigma):  # noqa: N802
    return separable(a, _sig(sigma, a.ndim), [0] * a.ndim)


def gaussianGradientMagnitude(a, sigma):  # noqa: N802
    nd, s = a.ndim, _sig(sigma, a.ndim)
    g = [separable(a, s, [1 if k == d else 0 for k in range(nd)]) for d in range(nd)]
    return np.sqrt(sum(x * x for x in g))


def laplacianOfGaussian(a, sigma):  # noqa: N802
    nd, s = a.ndim, _sig(sigma, a.ndim)
    return sum(separable(a, s, [2 if k == d else 0 for k in range(nd)]) for d in range(nd))


def _eig_desc(m):
    return np.linalg.eigvalsh(m)[..., ::-1]


def hessianOfGaussianEigenvalues(a, sigma):  # noqa: N802
    nd, s = a.ndim, _sig(sigma, a.ndim)
    h = np.zeros(a.shape + (nd, nd))
    for i in range(nd):
        for j in range(i, nd):
            o = [0] * nd
            o[i] += 1
            o[j] += 1
            h[..., i, j] = h[..., j, i] = separable(a, s, o)
    return _eig_desc(h)


def structureTensorEigenvalues(a, inner, outer=None):  # noqa: N802
    nd = a.ndim
    si = _sig(inner, nd)
    so = _sig(outer if outer is not None else [0.5 * v for v in si], nd)
    g = [separable(a, si, [1 if k == d else 0 for k in range(nd)]) for d in range(nd)]
    t = np.zeros(a.shape + (nd, nd))
    for i in range(nd):
        for j in range(i, nd):
            t[..., i, j] = t[..., j, i] = separable(g[i] * g[j], so, [0] * nd)
    return _eig_desc(t)


def differenceOfGaussians(a, sigma, sigma2=None):  # noqa: N802
    s2 = sigma2 if sigma2 is not None else [0.66 * v for v in _sig(sigma, a.ndim)]
    return gaussianSmoothing(a, sigma) - gaussianSmoothing(a, s2)
