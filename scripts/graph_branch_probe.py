"""Dev: do two branches of a captured HIP graph (a fork onto a second stream
and a join) run concurrently on this ROCm?  Times one spin kernel per branch
(torch.cuda._sleep), eager and captured, serial and forked."""
import torch


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3   # µs


def main():
    cyc = 200_000   # ≈ 80-100 µs per spin at the shader clock
    side = torch.cuda.Stream()

    def serial():
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)

    def forked():
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        main_s.wait_stream(side)

    one = timed(lambda: torch.cuda._sleep(cyc))
    print(f"one spin {one:.1f} us; eager serial {timed(serial):.1f}; eager forked {timed(forked):.1f}")
    for name, fn in (("serial", serial), ("forked", forked)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(4):
                    fn()
        torch.cuda.synchronize()
        print(f"graph {name}: {timed(g.replay) / 4:.1f} us per pair")


if __name__ == "__main__":
    main()
