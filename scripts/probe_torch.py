import os, sys
print("env", {k:v for k,v in os.environ.items() if any(s in k for s in ("HIP","ROCR","CUDA","HSA","GPU"))})
import torch
print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
sys.path.insert(0, os.getcwd())
from shadow_amd import Topology, synth, scenario
t = Topology(synth.ONE_GBIT_SWITCH_GML); scenario.register_hosts(t, 4); t.build_routes()
print("lib ok")
print("torch after", torch.cuda.is_available(), torch.cuda.device_count())
x = torch.ones(4, device="cuda"); print(x.sum().item())
