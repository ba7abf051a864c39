"""GPU filters of the filter-feature branch, with the ``fastfilters`` API.

The reference's BlockEdgeFeatures task, configured with ``filters`` and
``sigmas``, smooths each block's input with ``fastfilters`` (isotropic sigma)
or ``vigra.filters`` (per-axis sigma) through ``vu.apply_filter``
(utils/volume_utils.py:80-94) and accumulates every response channel over the
block's edges with ``ndist.accumulateInput``
(features/block_edge_features.py:151-168, 174-238).  This module provides the
filter names that code looks up with ``getattr(ff, filter_name)`` on the GPU:
separable Gaussian-derivative convolutions (``ctg_filter_conv_axis``, one
launch per axis), elementwise combines (``ctg_filter_combine``) and the
per-voxel symmetric eigenvalues (``ctg_sym_eigenvalues``), all in libctg.so.

Kernel rule (vigra ``initGaussian`` / ``initGaussianDerivative``
[UPSTREAM, unverified]): radius = int(3 sigma + 0.5 order + 0.5); taps
exp(-x^2 / 2 sigma^2) (times -x / sigma^2, or (x^2 / sigma^4 - 1 / sigma^2)
for the derivatives), normalised to sum 1 (smoothing), to a unit response to
f(x) = x (first derivative) or, after removing the DC part, to f(x) = x^2 / 2
(second derivative); borders mirror without repeating the edge voxel
(BORDER_TREATMENT_REFLECT).  fastfilters' own FIR implementation and its
defaults (structure-tensor outer scale, DoG ratio) are not in the image:
**parity unpinned** against both libraries; the tests pin this module to a
numpy/scipy restatement of the rule above.

Inputs are numpy arrays or CUDA tensors (2-D or 3-D, cast to float32);
results come back as numpy arrays for numpy inputs, tensors otherwise.
Multi-channel results (eigenvalues) are channel-last, descending, as
fastfilters returns them.
"""
from __future__ import annotations

import numpy as np

import ctypes

from . import _lib

__all__ = ['gaussianSmoothing', 'gaussianGradientMagnitude', 'laplacianOfGaussian', 'hessianOfGaussianEigenvalues',
           'structureTensorEigenvalues', 'differenceOfGaussians', 'gaussian_taps']


def gaussian_taps(sigma, order=0):
    """Correlation taps (out[p] = sum_k t[k] in[p + k - R]) of vigra's
    Gaussian (order 0) or Gaussian derivative (order 1, 2) kernel."""
    sigma = float(sigma)
    if sigma <= 0:
        if order != 0:
            raise ValueError('derivative filters need sigma > 0')
        return np.ones(1, np.float64)
    r = int(3.0 * sigma + 0.5 * order + 0.5)
    x = np.arange(-r, r + 1, dtype=np.float64)
    g = np.exp(-x * x / (2.0 * sigma * sigma))
    if order == 0:
        return g / g.sum()
    if order == 1:
        t = x / (sigma * sigma) * g              # correlation orientation: d/dx of f(x) = x is +1
        return t / np.sum(t * x)
    if order == 2:
        t = (x * x / sigma ** 4 - 1.0 / (sigma * sigma)) * g
        t -= t.mean()                            # no DC response
        return t / np.sum(t * x * x / 2.0)
    raise ValueError('order must be 0, 1 or 2')


def _torch():
    import torch
    return torch


def _as_device(x):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        t = x.to(dtype=torch.float32)
        if not t.is_cuda:
            t = t.cuda()
        return t.contiguous(), False
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    return torch.from_numpy(a).cuda(), True


def _sigmas(sigma, ndim):
    if isinstance(sigma, (tuple, list, np.ndarray)):
        s = [float(v) for v in sigma]
        if len(s) != ndim:
            raise ValueError('need one sigma per axis (%d), got %d' % (ndim, len(s)))
        return s
    return [float(sigma)] * ndim


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return _torch().cuda.current_stream().cuda_stream


def _conv(t, axis, taps):
    torch = _torch()
    out = torch.empty_like(t)
    w = np.ascontiguousarray(taps, dtype=np.float32)
    shape = np.asarray(t.shape, dtype=np.int64)
    _lib.check(_lib.load().ctg_filter_conv_axis(_ptr(t), _ptr(out), shape.ctypes.data, t.dim(), axis,
                                                w.ctypes.data, int(w.size), _stream()), 'conv_axis')
    return out


def _separable(t, sigmas, orders):
    """Apply the order-`orders[a]` Gaussian kernel along every axis a."""
    for a, (s, o) in enumerate(zip(sigmas, orders)):
        taps = gaussian_taps(s, o)
        if taps.size > 1:
            t = _conv(t, a, taps)
    return t


def _combine(op, a, b=None, c=None):
    torch = _torch()
    out = torch.empty_like(a)
    _lib.check(_lib.load().ctg_filter_combine(op, _ptr(a), _ptr(b), _ptr(c), _ptr(out), a.numel(),
                                              _stream()), 'combine')
    return out


def _eig(comps, dim):
    torch = _torch()
    stack = torch.stack(comps).contiguous()
    n = comps[0].numel()
    out = torch.empty(tuple(comps[0].shape) + (dim,), dtype=torch.float32, device=stack.device)
    _lib.check(_lib.load().ctg_sym_eigenvalues(_ptr(stack), dim, n, _ptr(out), _stream()), 'sym_eigenvalues')
    return out


def _ret(t, host):
    if host:
        _torch().cuda.synchronize()
        return t.cpu().numpy()
    return t


def _check_ndim(t):
    if t.dim() not in (2, 3):
        raise ValueError('filters take 2-D or 3-D arrays, got %d-D' % t.dim())


def gaussianSmoothing(array, sigma):  # noqa: N802
    t, host = _as_device(array)
    _check_ndim(t)
    return _ret(_separable(t, _sigmas(sigma, t.dim()), [0] * t.dim()), host)


def _gradient(t, sig):
    nd = t.dim()
    return [_separable(t, sig, [1 if a == d else 0 for a in range(nd)]) for d in range(nd)]


def gaussianGradientMagnitude(array, sigma):  # noqa: N802
    t, host = _as_device(array)
    _check_ndim(t)
    g = _gradient(t, _sigmas(sigma, t.dim()))
    return _ret(_combine(0, *g), host)


def laplacianOfGaussian(array, sigma):  # noqa: N802
    t, host = _as_device(array)
    _check_ndim(t)
    nd, sig = t.dim(), _sigmas(sigma, t.dim())
    dd = [_separable(t, sig, [2 if a == d else 0 for a in range(nd)]) for d in range(nd)]
    return _ret(_combine(1, *dd), host)


def _upper(nd):
    return [(a, b) for a in range(nd) for b in range(a, nd)]


def hessianOfGaussianEigenvalues(array, sigma):  # noqa: N802
    t, host = _as_device(array)
    _check_ndim(t)
    nd, sig = t.dim(), _sigmas(sigma, t.dim())
    comps = []
    for a, b in _upper(nd):
        orders = [0] * nd
        orders[a] += 1
        orders[b] += 1
        comps.append(_separable(t, sig, orders))
    return _ret(_eig(comps, nd), host)


def structureTensorEigenvalues(array, innerScale, outerScale=None):  # noqa: N802,N803
    """Eigenvalues of the Gaussian-smoothed (outerScale) outer product of the
    Gaussian gradient (innerScale); outerScale defaults to innerScale / 2
    (fastfilters' default is not in the image: parity unpinned)."""
    t, host = _as_device(array)
    _check_ndim(t)
    nd = t.dim()
    inner = _sigmas(innerScale, nd)
    outer = _sigmas(outerScale if outerScale is not None else
                    ([0.5 * s for s in inner] if isinstance(innerScale, (tuple, list)) else 0.5 * float(innerScale)),
                    nd)
    g = _gradient(t, inner)
    comps = [_separable(_combine(2, g[a], g[b]), outer, [0] * nd) for a, b in _upper(nd)]
    return _ret(_eig(comps, nd), host)


def differenceOfGaussians(array, sigma, sigma2=None):  # noqa: N802
    """G_sigma * f - G_sigma2 * f, sigma2 defaulting to 0.66 sigma (ilastik's
    ratio; parity unpinned)."""
    t, host = _as_device(array)
    _check_ndim(t)
    nd = t.dim()
    s1 = _sigmas(sigma, nd)
    s2 = _sigmas(sigma2 if sigma2 is not None else
                 ([0.66 * s for s in s1] if isinstance(sigma, (tuple, list)) else 0.66 * float(sigma)), nd)
    return _ret(_combine(3, _separable(t, s1, [0] * nd), _separable(t, s2, [0] * nd)), host)


def apply_filter(input_, filter_name, sigma, apply_in_2d=False):
    """vu.apply_filter (utils/volume_utils.py:80-94) on the GPU: per-axis
    sigma -> 3-D with that sigma; apply_in_2d -> per z-slice; else 3-D."""
    if isinstance(sigma, (tuple, list)) and apply_in_2d:
        raise ValueError('per-axis sigma is 3-D only (volume_utils.py:83-84)')
    filt = globals()[filter_name]
    if apply_in_2d and not isinstance(sigma, (tuple, list)):
        out = [filt(np.asarray(z), sigma) for z in np.asarray(input_)]
        return np.stack(out, axis=0)
    return filt(input_, sigma)
