import numpy as np
rng = np.random.default_rng(1)
def spd(n, dec):
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    ev = 10.0 ** (-dec * np.arange(n) / (n - 1))
    return (Q * ev) @ Q.T
def gj_elem(A):
    A = A.astype(np.float32).copy(); n = len(A)
    for p in range(n):
        piv = A[p, p]; pinv = np.float32(1) / piv
        e = A[p].copy(); e[p] = piv + np.float32(1)
        g = A[:, p] * pinv; g[p] = np.float32(1) - pinv
        A -= np.outer(g, e).astype(np.float32)
    return A
def gj_block(A, bs=16):
    A = A.astype(np.float32).copy(); n = len(A); nb = n // bs
    for k in range(nb):
        ks = slice(k*bs, (k+1)*bs)
        R = A[ks].copy()           # row block
        for p in range(bs):        # elimination on the row block
            col = k*bs + p
            piv = R[p, col]; pinv = np.float32(1) / piv
            e = R[p].copy(); e[col] = piv + np.float32(1)
            g = R[:, col] * pinv; g[p] = np.float32(1) - pinv
            R -= np.outer(g, e).astype(np.float32)
        for I in range(nb):
            if I == k: continue
            Is = slice(I*bs, (I+1)*bs)
            MIk = A[Is, ks].copy()
            for J in range(nb):
                if J == k: continue
                Js = slice(J*bs, (J+1)*bs)
                A[Is, Js] = A[Is, Js] - (MIk @ R[:, Js]).astype(np.float32)
            s = -1 if I < k else 1
            A[Is, ks] = -s * R[:, Is].T
        A[ks] = R
    return A
for dec in range(1, 7):
    A = spd(64, dec).astype(np.float32)
    A64 = A.astype(np.float64)
    for name, f in (("elem", gj_elem), ("block", gj_block)):
        X = f(A).astype(np.float64)
        print(dec, name, np.abs(A64 @ X - np.eye(64)).max())
def gj_block2(A, bs=16, colmode="explicit"):
    A = A.astype(np.float32).copy(); n = len(A); nb = n // bs
    for k in range(nb):
        ks = slice(k*bs, (k+1)*bs)
        R = A[ks].copy()
        for p in range(bs):
            col = k*bs + p
            piv = R[p, col]; pinv = np.float32(1) / piv
            e = R[p].copy(); e[col] = piv + np.float32(1)
            g = R[:, col] * pinv; g[p] = np.float32(1) - pinv
            R -= np.outer(g, e).astype(np.float32)
        for I in range(nb):
            if I == k: continue
            Is = slice(I*bs, (I+1)*bs)
            MIk = A[Is, ks].copy()
            for J in range(nb):
                if J == k: continue
                Js = slice(J*bs, (J+1)*bs)
                A[Is, Js] = A[Is, Js] - (MIk @ R[:, Js]).astype(np.float32)
            A[Is, ks] = -(MIk @ R[:, ks]).astype(np.float32)
        A[ks] = R
    return A
def gj_elem_rows_delayed(A, bs=16):
    # element GJ but rows outside the block updated with the partially-eliminated row block (rank-1 each pivot)
    return gj_elem(A)
print("explicit column update")
for dec in range(1, 7):
    A = spd(64, dec).astype(np.float32)
    X = gj_block2(A).astype(np.float64)
    print(dec, np.abs(A.astype(np.float64) @ X - np.eye(64)).max())
print("block size 4")
for dec in range(1, 7):
    A = spd(64, dec).astype(np.float32)
    X = gj_block(A, 4).astype(np.float64)
    print(dec, np.abs(A.astype(np.float64) @ X - np.eye(64)).max())
def gj_block3(A, bs=16):
    A = A.astype(np.float32).copy(); n = len(A); nb = n // bs
    for k in range(nb):
        ks = slice(k*bs, (k+1)*bs)
        P = gj_elem(A[ks, ks])
        T = (P @ A[ks]).astype(np.float32)
        for I in range(nb):
            if I == k: continue
            Is = slice(I*bs, (I+1)*bs)
            MIk = A[Is, ks].copy()
            for J in range(nb):
                if J == k: continue
                Js = slice(J*bs, (J+1)*bs)
                A[Is, Js] = A[Is, Js] - (MIk @ T[:, Js]).astype(np.float32)
            A[Is, ks] = -(MIk @ P).astype(np.float32)
        A[ks] = T
        A[ks, ks] = P
    return A
print("explicit P times row block, exact M_Ik")
for dec in range(1, 7):
    A = spd(64, dec).astype(np.float32)
    X = gj_block3(A).astype(np.float64)
    print(dec, np.abs(A.astype(np.float64) @ X - np.eye(64)).max())
