"""Synthetic SPD systems that feed the PCG hot path (host-side input plumbing).

These are the inputs of the reference's hot path, not part of it.  The
reference produces its matrices offline with ``datagen/*.py`` (pymathprim,
tetgen, pyssim -- none of which exist here), so every generator below is
either an exact restatement (``generate_spd_sparse_matrix``) or a stand-in
with the same structure, as SURVEY.md section 8(d) specifies:

* ``generate_spd_sparse_matrix``  -- restates ``datagen/synthetic.py:10-27``.
* ``poisson2d_grid``              -- stand-in for ``datagen/poisson.py:48-84``
  (cotangent Laplacian of a right-triangle grid, Dirichlet on a random 10 % of
  the boundary vertices, masked with ``neural_cg/data.py:159-170`` semantics).
* ``kuhn_laplacian``              -- the roofline target of SURVEY.md 8(d):
  Freudenthal/Kuhn tet grid, 14 neighbours + self per interior vertex.
* ``elasticity_box``              -- stand-in for ``datagen/elast_twist.py``:
  block_size 3 linear-elastic tet stiffness + mass/dt^2, Dirichlet x-ends.
* ``heat_tet``                    -- stand-in for ``datagen/heat_tetmesh.py``.
* ``heat_bunny``                  -- stand-in for ``datagen/heat.py`` on the bunny (C3).

All functions return scipy CSR matrices (float64, int32 indices, sorted) and,
where the reference has one, the Dirichlet mask ``[N, b]``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import scipy.sparse as sp


# ---------------------------------------------------------------------------
# datagen/synthetic.py:10-27
# ---------------------------------------------------------------------------
def generate_spd_sparse_matrix(n, sparsity=0.01, condition_amplifier=1e-6, random_state=None):
    """Random SPD ``MᵀM + αI`` exactly as ``datagen/synthetic.py:10-27``.

    ``random_state`` is forwarded to ``np.random.default_rng`` just like the
    reference (the datagen passes a ``np.random.RandomState``).
    """
    rng = np.random.default_rng(random_state)
    M = sp.random(n, n, density=sparsity, format="csr", random_state=rng)
    M.data = (M.data - 0.5) * 2
    scaling = np.linspace(1, condition_amplifier, n)
    D = sp.diags(scaling)
    M = D @ M
    A = M.T @ M
    A += sp.eye(n) * condition_amplifier
    return _canon(A)


def synthetic_c1(n: int = 10240, seed: int = 42):
    """BASELINE config 1: synthetic N=10240, sparsity 3e-4, amplifier 1e-5."""
    return generate_spd_sparse_matrix(n, 3e-4, 1e-5, np.random.RandomState(seed))


def _canon(A) -> sp.csr_matrix:
    A = sp.csr_matrix(A)
    A.sum_duplicates()
    A.sort_indices()
    A.indptr = A.indptr.astype(np.int32)
    A.indices = A.indices.astype(np.int32)
    return A


# ---------------------------------------------------------------------------
# Dirichlet masking (neural_cg/data.py:159-170 semantics)
# ---------------------------------------------------------------------------
def apply_dbc_masking(mat, mask: np.ndarray) -> sp.csr_matrix:
    """Zero rows/cols with ``mask == 0`` and put 1 on their diagonal.

    Same result as ``neural_cg/data.py:159-170`` (COO zeroing + ``diags(1-mask)``
    added through scipy's CSR addition, which drops explicit zeros).
    """
    coo = sp.coo_matrix(mat)
    m = np.asarray(mask, dtype=np.float64).ravel()
    data = coo.data.copy()
    data[m[coo.row] == 0] = 0
    data[m[coo.col] == 0] = 0
    coo = sp.coo_matrix((data, (coo.row, coo.col)), shape=coo.shape)
    out = coo.tocsr() + sp.diags(1.0 - m, 0, shape=coo.shape, format="csr")
    return _canon(out)


# ---------------------------------------------------------------------------
# Meshes
# ---------------------------------------------------------------------------
def grid_triangles(nx: int, ny: int) -> Tuple[np.ndarray, np.ndarray]:
    """Unit right-triangle grid with nx*ny vertices (row-major)."""
    xs, ys = np.meshgrid(np.arange(nx, dtype=np.float64), np.arange(ny, dtype=np.float64), indexing="xy")
    nodes = np.stack([xs.ravel(), ys.ravel()], axis=1)
    i, j = np.meshgrid(np.arange(nx - 1), np.arange(ny - 1), indexing="xy")
    v00 = (j * nx + i).ravel()
    v10 = v00 + 1
    v01 = v00 + nx
    v11 = v01 + 1
    tris = np.concatenate([np.stack([v00, v10, v11], 1), np.stack([v00, v11, v01], 1)], 0)
    return nodes, tris.astype(np.int64)


def cotangent_laplacian(nodes: np.ndarray, tris: np.ndarray) -> sp.csr_matrix:
    """Positive semi-definite cotangent Laplacian (stand-in for pymathprim.geometry.laplacian)."""
    n = nodes.shape[0]
    rows, cols, vals = [], [], []
    for k in range(3):
        a = tris[:, k]
        b = tris[:, (k + 1) % 3]
        c = tris[:, (k + 2) % 3]
        u = nodes[a] - nodes[c]
        v = nodes[b] - nodes[c]
        dot = np.sum(u * v, axis=1)
        if nodes.shape[1] == 2:
            cr = np.abs(u[:, 0] * v[:, 1] - u[:, 1] * v[:, 0])
        else:
            cr = np.linalg.norm(np.cross(u, v), axis=1)
        w = 0.5 * dot / cr  # 0.5 * cot(angle at c)
        rows += [a, b, a, b]
        cols += [b, a, a, b]
        vals += [-w, -w, w, w]
    L = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n)).tocsr()
    L.sum_duplicates()
    L.eliminate_zeros()
    return _canon(L)


def boundary_vertices_tri(tris: np.ndarray) -> np.ndarray:
    e = np.concatenate([tris[:, [0, 1]], tris[:, [1, 2]], tris[:, [2, 0]]], 0)
    e = np.sort(e, axis=1)
    uniq, cnt = np.unique(e, axis=0, return_counts=True)
    return np.unique(uniq[cnt == 1].ravel())


def poisson2d_grid(nx: int = 256, ny: int = 256, ratio: float = 0.1, seed: int = 42):
    """BASELINE config 2 stand-in: Poisson-2D, N = nx*ny (65,536 at 256²), fp64.

    Returns ``(A, mask[N,1], nodes)`` with A already Dirichlet-masked as
    ``datagen/poisson.py:74-81`` does.
    """
    nodes, tris = grid_triangles(nx, ny)
    L = cotangent_laplacian(nodes, tris)
    bnd = boundary_vertices_tri(tris)
    rng = np.random.default_rng(seed)
    dbc_cnt = int(ratio * len(bnd))
    dbc = rng.choice(bnd.shape[0], size=dbc_cnt, replace=False)
    mask = np.ones((L.shape[0], 1), dtype=np.float64)
    mask[bnd[dbc]] = 0
    return apply_dbc_masking(L, mask), mask, nodes


_KUHN_OFFSETS = np.array(
    [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1)], dtype=np.int64
)


def kuhn_laplacian(n: int = 101, shift: float = 1e-4, ny: Optional[int] = None, nz: Optional[int] = None):
    """Weighted graph Laplacian of the Kuhn (Freudenthal) tet grid + ``shift*I``.

    Vertex (i, j, k) -> (i*ny + j)*nz + k.  Every vertex couples to the 14
    Kuhn neighbours ±(1,0,0) ±(0,1,0) ±(0,0,1) ±(1,1,0) ±(1,0,1) ±(0,1,1)
    ±(1,1,1) with weight 1/|d|².  At n=101: N=1,030,301, nnz=15,210,901
    (SURVEY.md 8(d) roofline target).
    """
    nx = n
    ny = n if ny is None else ny
    nz = n if nz is None else nz
    N = nx * ny * nz
    rows, cols, vals = [], [], []
    idx = np.arange(N, dtype=np.int64).reshape(nx, ny, nz)
    deg = np.zeros(N, dtype=np.float64)
    for d in _KUHN_OFFSETS:
        w = 1.0 / float(np.dot(d, d))
        a = idx[: nx - d[0], : ny - d[1], : nz - d[2]].ravel()
        b = idx[d[0]:, d[1]:, d[2]:].ravel()
        rows += [a, b]
        cols += [b, a]
        vals += [np.full(a.size, -w), np.full(a.size, -w)]
        np.add.at(deg, a, w)
        np.add.at(deg, b, w)
    rows.append(np.arange(N))
    cols.append(np.arange(N))
    vals.append(deg + shift)
    A = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(N, N))
    return _canon(A)


def kuhn_tets(nx: int, ny: int, nz: int) -> Tuple[np.ndarray, np.ndarray]:
    """Vertices and tetrahedra of a Kuhn-split (6 tets / cube) box grid."""
    g = np.stack(np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij"), -1).reshape(-1, 3)
    nodes = g.astype(np.float64)
    idx = lambda i, j, k: (i * ny + j) * nz + k
    ci, cj, ck = np.meshgrid(np.arange(nx - 1), np.arange(ny - 1), np.arange(nz - 1), indexing="ij")
    ci, cj, ck = ci.ravel(), cj.ravel(), ck.ravel()
    tets = []
    import itertools

    for perm in itertools.permutations(range(3)):
        p = np.zeros((ci.size, 3), dtype=np.int64)
        v = [idx(ci, cj, ck)]
        for ax in perm:
            p[:, ax] += 1
            v.append(idx(ci + p[:, 0], cj + p[:, 1], ck + p[:, 2]))
        tets.append(np.stack(v, 1))
    return nodes, np.concatenate(tets, 0)


def _tet_gradients(nodes: np.ndarray, tets: np.ndarray):
    X = nodes[tets]  # [T,4,3]
    Dm = np.stack([X[:, 1] - X[:, 0], X[:, 2] - X[:, 0], X[:, 3] - X[:, 0]], -1)  # [T,3,3] columns
    vol = np.abs(np.linalg.det(Dm)) / 6.0
    Dinv = np.linalg.inv(Dm)  # rows = grads of barycentric 1..3
    g123 = Dinv  # [T,3(node),3(xyz)]
    g0 = -g123.sum(1, keepdims=True)
    return np.concatenate([g0, g123], 1), vol  # [T,4,3], [T]


def p1_stiffness(nodes, tets, kappa=None) -> sp.csr_matrix:
    G, vol = _tet_gradients(nodes, tets)
    w = vol if kappa is None else vol * kappa
    K = np.einsum("tad,tbd->tab", G, G) * w[:, None, None]
    r = np.repeat(tets, 4, axis=1).ravel()
    c = np.tile(tets, (1, 4)).ravel()
    n = nodes.shape[0]
    return _canon(sp.coo_matrix((K.ravel(), (r, c)), shape=(n, n)))


def lumped_mass(nodes, tets) -> np.ndarray:
    _, vol = _tet_gradients(nodes, tets)
    m = np.zeros(nodes.shape[0])
    np.add.at(m, tets.ravel(), np.repeat(vol / 4.0, 4))
    return m


def heat_tet(nx: int, ny: int, nz: int, rho: float = 2e-4, seed: int = 0):
    """Heat-tetmesh stand-in (``datagen/heat_tetmesh.py:26-56``): ``L + diag(M·ρ)``.

    Returns ``(A, mask[N,1], features[N,3])`` (features = xyz, as
    ``heat_tetmesh.py:99``).
    """
    nodes, tets = kuhn_tets(nx, ny, nz)
    rng = np.random.default_rng(seed)
    kappa = rng.uniform(0.01, 1.0, size=tets.shape[0])
    K = p1_stiffness(nodes, tets, kappa)
    M = lumped_mass(nodes, tets)
    A = sp.csr_matrix(K + sp.diags(M * rho))
    A.eliminate_zeros()
    A = _canon(A)
    mask = np.ones((A.shape[0], 1))
    return A, mask, nodes / max(nx, ny, nz)


MESH_DIR = __import__("pathlib").Path(__file__).resolve().parent / "meshes"


def gaussian_random_field(points: np.ndarray, seed: int, len_scale: float = 1.0, modes: int = 256) -> np.ndarray:
    """Seeded smooth random field at ``points`` (stand-in for ``gs.SRF(gs.Gaussian(dim=3, var=5,
    len_scale=1))`` of ``heat.py:47-48``; gstools is absent).  Randomised spectral sum over the
    Gaussian model's spectrum: the correlation ``exp(-π/4 (r/ℓ)²)`` has wave vectors
    ``k ~ N(0, (π/2)/ℓ² I)``.  The variance is irrelevant: ``heat.py:83-86`` renormalises."""
    rng = np.random.default_rng(seed)
    k = rng.normal(scale=np.sqrt(np.pi / 2) / len_scale, size=(modes, points.shape[1]))
    phi = rng.uniform(0, 2 * np.pi, size=modes)
    return np.sqrt(2.0 / modes) * np.cos(points @ k.T + phi).sum(1)


def heat_bunny(seed: int = 42, var: float = 0.99, eps: float = 1e-4, dirichlet: float = 0.05):
    """BASELINE config 3 stand-in (``datagen/heat.py:22-96`` on ``bunny_low_res.obj``).

    Mesh: Kuhn split (6 tets / cell) of every grid cell whose 8 corners lie inside the bunny
    (``meshes/bunny_grid.npz``: winding-number voxelisation of the .obj, written by
    ``tests/golden/make_golden.py bunny``) -- 6.3 k vertices against the reference's tetgen 6276.
    Operator: ``L(κ_tet) + eps·M_lumped`` with ``κ_tet`` the per-tet mean (``to_tet_field``,
    ``heat.py:15-19``) of a field renormalised as ``heat.py:83-86``.  Dirichlet: the lowest
    ``dirichlet`` fraction of vertices by height (the reference's heat data has none; SURVEY 8(d)
    adds them so the masked assembly is exercised).  Features: ``[field, x, y, z]`` -- the step's
    field (``heat.py:96``) then the shared xyz (``:75-76``); make_data appends the mask: F_in = 5.

    Returns ``(A_raw, mask[N,1], features[N,4])``.
    """
    z = np.load(MESH_DIR / "bunny_grid.npz")
    ins = z["inside"]
    h = float(z["h"])
    nx, ny, nz = ins.shape
    cell = np.ones((nx - 1, ny - 1, nz - 1), dtype=bool)
    for a in (0, 1):
        for b in (0, 1):
            for c in (0, 1):
                cell &= ins[a:nx - 1 + a, b:ny - 1 + b, c:nz - 1 + c]
    nodes, tets = kuhn_tets(nx, ny, nz)
    tets = tets.reshape(6, (nx - 1) * (ny - 1) * (nz - 1), 4)[:, cell.ravel()].reshape(-1, 4)
    used, tets = np.unique(tets, return_inverse=True)
    tets = tets.reshape(-1, 4)
    nodes = z["lo"][None, :] + h * nodes[used]
    field = gaussian_random_field(nodes, seed)
    field = field - field.min()
    field = field / (field.max() + 1e-4)
    field = field * var + (1 - var)
    K = p1_stiffness(nodes, tets, field[tets].mean(1))
    A = _canon(K + sp.diags(eps * lumped_mass(nodes, tets)))
    mask = np.ones((A.shape[0], 1))
    mask[np.argsort(nodes[:, 1], kind="stable")[: int(dirichlet * A.shape[0])]] = 0.0
    return A, mask, np.concatenate([field[:, None], nodes], 1)


def elasticity_box(nx: int = 117, ny: int = 30, nz: int = 30, E: float = 3e6, nu: float = 0.4,
                   density: float = 1.0, dt: float = 0.01):
    """Elasticity-twist stand-in, block_size 3 (``datagen/elast_twist.py:17-129``).

    Linear-elastic P1 tet stiffness (E, ν) + lumped mass/dt², vertices at
    both x-ends Dirichlet.  Returns ``(A_bsr_pattern_csr, mask[N,3], nodes)``
    where A is the *scalar* CSR (n = 3N) before masking and mask is per dof.
    """
    nodes, tets = kuhn_tets(nx, ny, nz)
    nodes = nodes / float(max(ny, nz) - 1)
    G, vol = _tet_gradients(nodes, tets)
    lam = E * nu / ((1 + nu) * (1 - 2 * nu))
    mu = E / (2 * (1 + nu))
    # K_ab(ij) = vol * (lam * g_a,i g_b,j + mu * (g_a,j g_b,i + δ_ij g_a·g_b))
    gg = np.einsum("tad,tbd->tab", G, G)
    Kt = (lam * np.einsum("tai,tbj->tabij", G, G)
          + mu * np.einsum("taj,tbi->tabij", G, G)
          + mu * gg[:, :, :, None, None] * np.eye(3)[None, None, None])
    Kt *= vol[:, None, None, None, None]
    T = tets.shape[0]
    ra = (3 * tets[:, :, None, None, None] + np.arange(3)[None, None, None, :, None])
    cb = (3 * tets[:, None, :, None, None] + np.arange(3)[None, None, None, None, :])
    ra = np.broadcast_to(ra, (T, 4, 4, 3, 3)).ravel()
    cb = np.broadcast_to(cb, (T, 4, 4, 3, 3)).ravel()
    n = 3 * nodes.shape[0]
    K = sp.coo_matrix((Kt.ravel(), (ra, cb)), shape=(n, n)).tocsr()
    m = lumped_mass(nodes, tets) * density / dt ** 2
    A = _canon(K + sp.diags(np.repeat(m, 3)))
    mask = np.ones((nodes.shape[0], 3))
    x = nodes[:, 0]
    mask[(x <= x.min() + 1e-9) | (x >= x.max() - 1e-9)] = 0
    return A, mask, nodes


# ---------------------------------------------------------------------------
# Block (graph) view of a scalar CSR, the reference's edge_index / block_values
# ---------------------------------------------------------------------------
@dataclass
class BlockGraph:
    """COO block view of a matrix (``neural_cg/data.py:471-572`` ``load``).

    ``edge_index [2,E]`` int64 row-major sorted, ``block_values [E,b,b]`` f64,
    ``num_nodes`` = block rows.
    """

    edge_index: np.ndarray
    block_values: np.ndarray
    num_nodes: int
    block_size: int


def to_block_graph(A: sp.csr_matrix, block_size: int = 1) -> BlockGraph:
    if block_size == 1:
        coo = sp.coo_matrix(A)
        return BlockGraph(np.vstack([coo.row, coo.col]).astype(np.int64),
                          coo.data.astype(np.float64).reshape(-1, 1, 1), A.shape[0], 1)
    bsr = sp.bsr_matrix(sp.csr_matrix(A), blocksize=(block_size, block_size))
    bsr.sort_indices()
    nb = A.shape[0] // block_size
    rows = np.repeat(np.arange(nb), np.diff(bsr.indptr))
    return BlockGraph(np.vstack([rows, bsr.indices]).astype(np.int64), bsr.data.astype(np.float64),
                      nb, block_size)


def kuhn_dirichlet(n: int = 101, shift: float = 1e-4):
    """Bench workload: ``kuhn_laplacian(n)`` with Dirichlet vertices on the i = 0 face.

    Returns ``(A_raw, mask[N,1])``; masking is applied by the hot path's own assembly
    (``to_csr_cpu`` semantics), like ``infer.py:282`` does for every sample.
    """
    A = kuhn_laplacian(n, shift)
    mask = np.ones((A.shape[0], 1), dtype=np.float64)
    mask[: n * n] = 0.0  # vertex index (i*n + j)*n + k with i = 0
    return A, mask


def renumber(A: sp.csr_matrix, mask: np.ndarray, order: str, seed: int = 0, return_perm: bool = False):
    """``A`` and ``mask`` under a symmetric renumbering (P A Pᵀ, P mask): ``"rand"`` = a seeded random
    permutation (no locality at all), ``"rcm"`` = that random permutation followed by reverse
    Cuthill-McKee (scipy.sparse.csgraph) -- a banded but irregular ordering like an RCM-ordered
    tet mesh's, with many distinct row-relative offsets per 64-row slice.  Same matrix, same nnz."""
    from scipy.sparse.csgraph import reverse_cuthill_mckee

    n = A.shape[0]
    perm = np.random.default_rng(seed).permutation(n)
    if order == "rcm":
        Ar = sp.csr_matrix(A)[perm][:, perm]
        perm = perm[reverse_cuthill_mckee(sp.csr_matrix(Ar), symmetric_mode=True)]
    elif order != "rand":
        raise ValueError(order)
    B = sp.csr_matrix(sp.csr_matrix(A)[perm][:, perm])
    B.sort_indices()
    if return_perm:
        return B, mask[perm], perm
    return B, mask[perm]


# ---------------------------------------------------------------------------
# Unstructured tet meshes (datagen/heat_tetmesh.py on tetgen meshes)
# ---------------------------------------------------------------------------
def delaunay_tets(n_pts: int, seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Unstructured tet mesh of the unit cube with about ``n_pts`` vertices: the 3-D Delaunay
    triangulation (scipy.spatial / qhull) of a seeded UNIFORM random point cloud -- no lattice, so no
    stencil: vertex degrees vary (rows of 4 to ~35 entries, ~15.7 on average), like the tetgen meshes
    the reference's heat data come from (``neural_cg/datagen_helper.py:113-137``, 400-32 k vertices,
    ``preprocess/msh_to_npy.py:77-86``).  The cloud fills a box one mean spacing h = n^(-1/3) larger
    than the cube on every side and only the tets with all four vertices inside the cube are kept: the
    hull's flat slivers (4 nearly coplanar points on a face, stiffness entries ~1e5 x the median) never
    enter, interior tets keep the diagonal within ~35 x its median.  Vertices are numbered by a spatial
    bucket sort (cells of size h, x slowest, z fastest; the cell's points by x), the locality-preserving
    numbering a meshing tool emits; ``renumber`` gives the irregular ones.  Only elementwise numpy
    and qhull: the same bits on every host (tests pin A's sha256)."""
    from scipy.spatial import Delaunay

    h = float(n_pts) ** (-1.0 / 3.0)
    n_gen = int(round(n_pts * (1.0 + 2.0 * h) ** 3))
    rng = np.random.default_rng(seed)
    pts = rng.uniform(-h, 1.0 + h, size=(n_gen, 3))
    tets = Delaunay(pts).simplices.astype(np.int64)
    inside = np.all((pts >= 0.0) & (pts <= 1.0), axis=1)
    tets = tets[inside[tets].all(axis=1)]
    used = np.unique(tets)
    cells = np.minimum((pts[used] / h).astype(np.int64), int(1.0 / h) + 1)
    m = int(cells.max()) + 1
    key = (cells[:, 0] * m + cells[:, 1]) * m + cells[:, 2]
    order = np.lexsort((pts[used, 0], key))  # by cell, then x inside the cell
    new = np.empty(n_gen, dtype=np.int64)
    new[used[order]] = np.arange(used.size)
    tets = new[tets]
    # orient every tet positively (det > 0): swap its last two vertices where needed
    nodes = pts[used[order]]
    d = _tet_dets(nodes, tets)
    neg = d < 0
    tets[neg, 2], tets[neg, 3] = tets[neg, 3].copy(), tets[neg, 2].copy()
    return nodes, tets


def _tet_dets(nodes: np.ndarray, tets: np.ndarray) -> np.ndarray:
    X = nodes[tets]
    a, b, c = X[:, 1] - X[:, 0], X[:, 2] - X[:, 0], X[:, 3] - X[:, 0]
    return (a[:, 0] * (b[:, 1] * c[:, 2] - b[:, 2] * c[:, 1]) - a[:, 1] * (b[:, 0] * c[:, 2] - b[:, 2] * c[:, 0])
            + a[:, 2] * (b[:, 0] * c[:, 1] - b[:, 1] * c[:, 0]))


def p1_laplacian_exact(nodes: np.ndarray, tets: np.ndarray) -> Tuple[sp.csr_matrix, np.ndarray]:
    """P1 stiffness (cotangent Laplacian, ``pymathprim.geometry.laplacian`` as heat_tetmesh.py:26
    calls it) and the lumped mass (``lumped_mass``, :27) of a positively oriented tet mesh, with
    explicit cofactor arithmetic only (no LAPACK / BLAS, so the bits do not depend on the host's
    BLAS kernels): grad λ_a = cofactor row / det, K_ab += vol · (g_a · g_b), M_a += vol / 4."""
    X = nodes[tets]
    a, b, c = X[:, 1] - X[:, 0], X[:, 2] - X[:, 0], X[:, 3] - X[:, 0]
    cross = lambda u, v: np.stack([u[:, 1] * v[:, 2] - u[:, 2] * v[:, 1], u[:, 2] * v[:, 0] - u[:, 0] * v[:, 2],
                                   u[:, 0] * v[:, 1] - u[:, 1] * v[:, 0]], 1)
    bc, ca, ab = cross(b, c), cross(c, a), cross(a, b)
    det = a[:, 0] * bc[:, 0] + a[:, 1] * bc[:, 1] + a[:, 2] * bc[:, 2]
    g1, g2, g3 = bc / det[:, None], ca / det[:, None], ab / det[:, None]
    g0 = -(g1 + g2 + g3)
    G = np.stack([g0, g1, g2, g3], 1)  # [T, 4, 3]
    vol = det / 6.0
    K = (G[:, :, None, 0] * G[:, None, :, 0] + G[:, :, None, 1] * G[:, None, :, 1]
         + G[:, :, None, 2] * G[:, None, :, 2]) * vol[:, None, None]
    n = nodes.shape[0]
    r = np.repeat(tets, 4, axis=1).ravel()
    cidx = np.tile(tets, (1, 4)).ravel()
    S = _canon(sp.coo_matrix((K.ravel(), (r, cidx)), shape=(n, n)))
    S = _canon(sp.triu(S) + sp.triu(S, 1).T)  # exactly symmetric (duplicate sums run in sort order)
    mass = np.bincount(tets.ravel(), weights=np.repeat(vol / 4.0, 4), minlength=n)
    return S, mass


def smooth_random_field(points: np.ndarray, seed: int, cells: int = 4) -> np.ndarray:
    """Seeded smooth random field (stand-in for heat_tetmesh.py:29-31's gstools Gaussian SRF; gstools
    is absent): trilinear interpolation of uniform random values on a ``cells``³ lattice over the
    points' bounding box -- additions and multiplications only, so host-independent bits."""
    rng = np.random.default_rng(seed)
    v = rng.uniform(0.0, 1.0, size=(cells + 1,) * 3)
    lo = points.min(0)
    span = np.maximum(points.max(0) - lo, 1e-300)
    u = (points - lo) / span * cells
    i = np.minimum(u.astype(np.int64), cells - 1)
    f = u - i
    out = np.zeros(points.shape[0])
    for dx in (0, 1):
        wx = f[:, 0] if dx else 1.0 - f[:, 0]
        for dy in (0, 1):
            wy = f[:, 1] if dy else 1.0 - f[:, 1]
            for dz in (0, 1):
                wz = f[:, 2] if dz else 1.0 - f[:, 2]
                out += wx * wy * wz * v[i[:, 0] + dx, i[:, 1] + dy, i[:, 2] + dz]
    return out


def delaunay_heat(n_pts: int, seed: int = 0, min_density: float = 1e-4, max_density: float = 5e-4,
                  dirichlet: bool = True):
    """Heat on an unstructured Delaunay tet mesh, ``datagen/heat_tetmesh.py:17-56``: ``S = L +
    diag(M · ρ)`` with ``L`` the P1 Laplacian, ``M`` the lumped mass and ``ρ`` a smooth random field
    renormalised into [min_density, max_density] (config/heat_tetmesh.yaml: 1e-4, 5e-4) as
    heat_tetmesh.py:32-34 does.  Dirichlet (``dirichlet``): the vertices within one mean spacing of
    the x = 0 face (mask 0; heat_tetmesh has none -- SURVEY 8(d) adds them so the masked assembly
    runs).  Node features = xyz (heat_tetmesh.py:99 returns the nodes); make_data appends the mask.

    Returns ``(A_raw, mask[N,1], features[N,3])``."""
    nodes, tets = delaunay_tets(n_pts, seed)
    S, mass = p1_laplacian_exact(nodes, tets)
    field = smooth_random_field(nodes, seed + 1)
    field = field - field.min()
    field = field / (field.max() + 1e-4)
    field = field * (max_density - min_density) + min_density
    A = _canon(S + sp.diags(mass * field))
    mask = np.ones((A.shape[0], 1))
    if dirichlet:
        mask[nodes[:, 0] < float(n_pts) ** (-1.0 / 3.0)] = 0.0
    return A, mask, nodes


def matrix_sha256(A: sp.csr_matrix) -> str:
    """sha256 of a CSR matrix's (indptr int64, indices int64, data float64) bytes."""
    import hashlib

    h = hashlib.sha256()
    for arr, dt in ((A.indptr, np.int64), (A.indices, np.int64), (A.data, np.float64)):
        h.update(np.ascontiguousarray(arr, dtype=dt).tobytes())
    return h.hexdigest()


def _count(tok: str) -> int:
    """'1m' -> 1,000,000, '64k' -> 64,000, '5000' -> 5,000."""
    mult = {"k": 1000, "m": 1000000}.get(tok[-1:], 1)
    return int(tok[:-1] if mult > 1 else tok) * mult


def workload(name: str):
    """Named systems: returns ``(A_raw, mask, node_features, block_size, edge_to_node)``.

    ``kuhn<N>`` is the structured Kuhn-tet grid (N³ vertices, Dirichlet face); ``kuhn<N>rcm`` and
    ``kuhn<N>rand`` are the same system renumbered (``renumber``): irregular orderings of the same
    1M-row problem.  ``delaunay<N>`` (``delaunay1m``, ``delaunay64k``, ...) is the unstructured
    Delaunay heat system of about N vertices (``delaunay_heat``: the shape of the reference's tetgen
    meshes, datagen/heat_tetmesh.py), ``delaunay<N>rcm`` / ``rand`` its renumberings."""
    import re

    m = re.fullmatch(r"kuhn(\d*)(rcm|rand)?", name)
    if m:
        n = int(m.group(1) or 101)
        A, mask = kuhn_dirichlet(n)
        if m.group(2):
            A, mask = renumber(A, mask, m.group(2))
        return A, mask, None, 1, "disable"
    m = re.fullmatch(r"delaunay(\d+[km]?)(rcm|rand)?", name)
    if m:
        A, mask, nodes = delaunay_heat(_count(m.group(1)))
        if m.group(2):
            A, mask, perm = renumber(A, mask, m.group(2), return_perm=True)
            nodes = nodes[perm]
        return A, mask, nodes, 1, "disable"
    if name.startswith("poisson"):
        n = int(name[7:] or 256)
        A, mask, _ = poisson2d_grid(n, n)
        return A, mask, None, 1, "disable"
    if name.startswith("synthetic"):
        n = int(name[9:] or 10240)
        return synthetic_c1(n), None, None, 1, "mean"
    if name == "bunny":
        A, mask, feats = heat_bunny()
        return A, mask, feats, 1, "disable"
    if name.startswith("elast"):
        A, mask, nodes = elasticity_box()
        return A, mask, np.concatenate([nodes, np.zeros_like(nodes)], 1), 3, "disable"
    raise KeyError(name)
