"""Which ATen ops launch kernels inside one BERT-base (or ResNet-50) training step:
torch.profiler over 2 steps after warm-up, CUDA time per (op, input shapes),
kernel-launching ops only.  Used to find the framework ops left in the step."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.trainer.engine import Engine, init_distributed  # noqa: E402


def main() -> None:
    which = sys.argv[1] if len(sys.argv) > 1 else "bert"
    info = init_distributed()
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(0)
    if which == "bert":
        from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch
        cfg = BertConfig.base()
        model = BertForPreTraining(cfg)
        batch = synthetic_mlm_batch(cfg, 256, 128, g, info.device)
        eng = Engine(model, bert_loss, optimizer="adam", lr=1e-4, weight_decay=0.01, dist_info=info, channels_last=False)
    else:
        from kubeflow_controller_amd.models.resnet import ResNet
        from kubeflow_controller_amd.ops.loss import cross_entropy
        model = ResNet(layers=(3, 4, 6, 3), num_classes=1000)
        x = torch.randn(256, 3, 224, 224, device=info.device, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (256,), device=info.device)
        batch = (x, y)
        eng = Engine(model, lambda m, a, b: cross_entropy(m(a), b), optimizer="sgd", lr=0.1, dist_info=info)
    for _ in range(4):
        eng.train_step(*batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(2):
            eng.train_step(*batch)
        torch.cuda.synchronize()
    rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::") and e.device_time_total > 0]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:25]:
        print(f"{e.self_device_time_total / 2:9.1f} us/step  x{e.count // 2:<3d} {e.key:28s} {str(e.input_shapes)[:110]}")


if __name__ == "__main__":
    main()
