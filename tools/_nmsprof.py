import sys, torch
sys.path.insert(0, '/root/repo')
from edgeml_amd import models, synthetic
m = models.ssdlite320_mobilenet_v3_large().to("cuda")
m.CHAINS = 1
p = m.plan(16, 640, 640)
p.input.tensor().copy_(synthetic.make_batch(16, 640, 640, seed=3).cuda())
for _ in range(3):
    p.run()
torch.cuda.synchronize()
print("counts", p.out_count.tensor().cpu().tolist()[:4])
