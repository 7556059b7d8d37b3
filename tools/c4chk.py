import sys, os, time
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests", "golden"))
import torch, bench
dev = torch.device("cuda:0")
wl = bench.Nested(1 << 25, 0, dev)
print("arena-wire mod16", (wl.arena.data_ptr() - wl.wire.data_ptr()) % 16, "arena", wl.arena.numel(), "wire", wl.wire.numel(), flush=True)
for k in range(5):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    wl.timed_step(ev); torch.cuda.synchronize()
    print("enc %.3f dec %.3f" % (ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])), flush=True)
for k in range(4):
    wl.encode(); torch.cuda.synchronize(); time.sleep(0.05)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); wl.decode(); e1.record(); torch.cuda.synchronize()
    print("isolated dec %.3f" % e0.elapsed_time(e1), flush=True)
for k in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); wl.decode(); e1.record(); torch.cuda.synchronize()
    print("back-to-back dec %.3f" % e0.elapsed_time(e1), flush=True)
