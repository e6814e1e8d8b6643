"""Does hipExtStreamCreateWithCUMask restrict work here?  A compute-bound matmul loop on a stream masked
to half / a quarter of the CUs vs an unmasked stream (ms per loop)."""
import ctypes, time, torch
hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(0).multi_processor_count
def masked(bits):
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), words)
    print("create rc", rc, "words", [hex(w) for w in words], flush=True)
    return torch.cuda.ExternalStream(h.value)
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
cfgs = [("full", torch.cuda.Stream()), ("alt-bits", masked(range(0, NCU, 2))), ("first64", masked(range(64))),
        ("first128", masked(range(128))), ("last128", masked(range(128, 256))),
        ("even-words", masked([i for i in range(NCU) if (i // 32) % 2 == 0])),
        ("low16-each-word", masked([i for i in range(NCU) if i % 32 < 16])),
        ("low24-each-word", masked([i for i in range(NCU) if i % 32 < 24])),
        ("hi8-each-word", masked([i for i in range(NCU) if i % 32 >= 24]))]
for name, s in cfgs:
    with torch.cuda.stream(s):
        for rep in range(2):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            for _ in range(10):
                b = a @ a
            torch.cuda.synchronize()
        print(name, f"{(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
