import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
order = sys.argv[1]
import torch
import rgbd360_amd as R
if order == "torch_first":
    x = torch.ones(4, device="cuda:0"); torch.cuda.synchronize(); print("torch ok", x.sum().item())
    c = R.Context(0); print("r360 ok")
else:
    c = R.Context(0); print("r360 ok")
    x = torch.ones(4, device="cuda:0"); torch.cuda.synchronize(); print("torch ok", x.sum().item())
