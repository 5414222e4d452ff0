import sys, torch, json
sys.path.insert(0, '.')
import fem355
from fem355 import element, mesh, system
dev = torch.device('cuda', 0)
out = {}
for et, gen, n in (("c3d8", mesh.hex_box, 30), ("c3d6", mesh.wedge_box, 25), ("c3d10", mesh.tet10_cube, 16)):
    c, el = gen(n, jitter=0.1, device=dev)
    K = element.compute_K_matrix(c, el, et, 113.8e9, 0.342, device=dev, dtype=torch.float64)
    g = system.build_graph(el, c.shape[0])
    for bs in (3, 1):
        Kb = K if bs == 3 else K[:, 0::3, 0::3].contiguous()
        A = system.SellMatrix(g, bs).add_element_matrices(Kb, el)
        out[f"{et}_bs{bs}"] = int(A.vals.view(torch.int64).sum())
print(json.dumps(out))
