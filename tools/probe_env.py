"""Environment probe for the GPU box: device props, torch path step time, graph capture."""
import json, time, sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = {}
out["torch"] = torch.__version__
out["hip"] = torch.version.hip
out["dev"] = torch.cuda.get_device_name(0)
p = torch.cuda.get_device_properties(0)
out["cus"] = p.multi_processor_count
out["mem_gb"] = p.total_memory / 2**30
out["gcn"] = getattr(p, "gcnArchName", "")
from gfedntm_amd.data.synthetic import generate_synthetic, node_vocabulary_terms, remap_to_vocabulary
from gfedntm_amd.data.vocab import union_vocabulary, vocabulary_dict
from gfedntm_amd.data.bow import BOWDataset, DeviceCSR, BatchPlan
from gfedntm_amd.models import AVITM
c = generate_synthetic(vocab_size=5000, n_topics=50, n_docs=1000, n_nodes=1, frozen_topics=5, seed=1)
terms = union_vocabulary([node_vocabulary_terms(c, 0)])
voc = vocabulary_dict(terms)
X = remap_to_vocabulary(c, 0, voc)
m = AVITM(input_size=len(terms), n_components=50, hidden_sizes=(50, 50), verbose=False, backend="torch")
data = DeviceCSR(X, "cuda")
plan = BatchPlan.build(data.n_docs, 64, 400, seed=0)
m.engine.bind_data(data, plan)
for s in range(50):
    m.engine.step(s)
torch.cuda.synchronize()
t = time.perf_counter()
for s in range(50, 400):
    m.engine.step(s)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 350
out["torch_step_ms"] = dt * 1e3
out["torch_docs_per_s"] = 64 / dt
# graph capture smoke
x = torch.randn(64, 64, device="cuda")
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    y = x @ x
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    y = x @ x
g.replay(); torch.cuda.synchronize()
out["graph_ok"] = True
print(json.dumps(out))
