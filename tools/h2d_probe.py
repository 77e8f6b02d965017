"""Host-input costs of fri_commit on the GPU box (DESIGN §8 PCIe-inclusive):
pageable hipMemcpy, hipHostRegister + copy + unregister, pinned copy, and a
vectorised host scan of the same 8 MiB of coefficients.  Run through gpurun."""
import ctypes, time
import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
P = 3221225473
d = 1 << 21
a = (np.random.default_rng(1).integers(0, P, d, dtype=np.uint64)).astype(np.uint32)
dev = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(4 * d)) == 0
H2D = 1


def t(f, reps=20):
    f()
    hip.hipDeviceSynchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        hip.hipDeviceSynchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


src = a.ctypes.data_as(ctypes.c_void_p)
print("pageable hipMemcpy      %.3f ms" % t(lambda: hip.hipMemcpy(dev, src, ctypes.c_size_t(4 * d), H2D)))


def reg():
    assert hip.hipHostRegister(src, ctypes.c_size_t(4 * d), 0) == 0
    hip.hipMemcpy(dev, src, ctypes.c_size_t(4 * d), H2D)
    hip.hipHostUnregister(src)


print("register+copy+unreg     %.3f ms" % t(reg))
pin = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(pin), ctypes.c_size_t(4 * d), 0) == 0
ctypes.memmove(pin, src, 4 * d)
print("pinned hipMemcpy        %.3f ms" % t(lambda: hip.hipMemcpy(dev, pin, ctypes.c_size_t(4 * d), H2D)))
print("memmove to pinned       %.3f ms" % t(lambda: ctypes.memmove(pin, src, 4 * d)))
print("numpy max scan          %.3f ms" % t(lambda: int(a.max()) < P))
