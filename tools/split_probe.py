"""Probe: one 512-frame extraction vs the same frames as 2 x 256 (or 4 x 128)
sub-batches on separate streams (kernel tails and the octree's short level
workgroups filled by the other sub-batch).  Prints ms per 512 frames."""
import sys, time
sys.path.insert(0, "orb-slam2-annotation_amd")
import torch
import orbgpu, synth

W, H, NF, B = 640, 480, 1000, 512
dev = torch.device("cuda:0")
pitch = (W + 15) // 16 * 16
frames = synth.torch_stream(B, W, H, device=dev, pitch=pitch, bounded=True)
for nsplit in (1, 2, 4, 1, 2):
    sb = B // nsplit
    exs = [orbgpu.Extractor(nfeatures=NF, width=W, height=H, max_batch=sb) for _ in range(nsplit)]
    cap = exs[0].max_keypoints
    sts = [torch.cuda.Stream(dev, priority=-1) for _ in range(nsplit)]
    outs = [(torch.zeros((sb, cap, 7), dtype=torch.float32, device=dev),
             torch.zeros((sb, cap, 32), dtype=torch.uint8, device=dev),
             torch.zeros(sb, dtype=torch.int32, device=dev)) for _ in range(nsplit)]

    def run():
        for i in range(nsplit):
            exs[i].extract_batch(frames[i * sb:(i + 1) * sb], *outs[i], stream=sts[i], row_step=pitch,
                                 frame_step=pitch * H)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    for i in range(nsplit):
        exs[i].sync(sts[i])
    print(f"split {nsplit}: {dt:.3f} ms per {B} frames, {B / dt * 1e3:.0f} frames/s, kp {outs[0][2].float().mean().item():.1f}", flush=True)
