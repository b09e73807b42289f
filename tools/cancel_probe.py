"""Diagnostic: time a cancelled DirectLighting frame (tests/test_cancel.py's
DL case) phase by phase. Run under rocprofv3 --kernel-trace to see which
kernels still run after the cancel."""
import sys
import threading
import time

sys.path.insert(0, "go-pbrt_amd")
import pbrtgpu as G  # noqa: E402
from pbrtgpu import abi  # noqa: E402

sc = G.Scene.cornell(1920, 1080)
dl = dict(integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)
side = int(sys.argv[1]) if len(sys.argv) > 1 else 0
with G.Renderer(sc) as r:
    t0 = time.time()
    r.render(abi.render_desc(8, 8, **dl))
    t8 = time.time() - t0
    if not side:
        side = 8
        while side < 128 and t8 * (side / 8) ** 2 < 1.0:
            side *= 2
    print(f"t8={t8:.3f}s side={side}", flush=True)
with G.Renderer(sc) as r:
    ta = time.time()
    r.render_async(abi.render_desc(side, side, **dl))
    tb = time.time()
    fired = []
    tm = threading.Timer(0.1, lambda: (fired.append(time.time()), G.lib().pbrt_gpu_cancel(r.h)))
    tm.start()
    try:
        st = r.synchronize()
        print("not cancelled", st.kernel_ms)
    except G.PbrtError as e:
        print("cancelled rc", e.code)
    te = time.time()
    tm.join()
    print(f"render_async {tb - ta:.3f}s, cancel at +{fired[0] - tb:.3f}s, done {te - fired[0]:.3f}s after cancel",
          flush=True)
