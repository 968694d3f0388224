"""Child of test_cu_split.py: apply MDT_CU_SPLIT before HIP initialises,
then report how many distinct CUs a 4096-workgroup probe grid ran on."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from multidisttorch_amd.runtime.env import apply_cu_split

    mask = apply_cu_split()
    import torch

    from multidisttorch_amd.ops import native

    C = native.require()
    out = torch.zeros(4096, dtype=torch.int32, device="cuda")
    C.probe_cu_ids(out)
    torch.cuda.synchronize()
    ids = set(out.cpu().tolist())
    print("RESULT " + json.dumps({"mask": mask, "distinct_cus": len(ids)}), flush=True)


if __name__ == "__main__":
    main()
