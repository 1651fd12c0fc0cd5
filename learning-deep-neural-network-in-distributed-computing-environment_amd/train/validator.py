"""Validation and test evaluation.

validate():  eval + no_grad over the rank's validation shard -> (mean batch loss,
             accuracy %)                              BAR/validator.py:3-23
evaluate():  rank-0 test pass -> (loss, accuracy %, preds, labels) and
             precision / recall / F1 with macro, weighted and micro averaging,
             printed like BAR/evaluator.py:41-59 -- computed on the device from a
             confusion matrix (no per-batch host copies, no sklearn needed).

Loss and correct counts accumulate on the device; one host sync per pass.
"""
from __future__ import annotations

import torch

from ..models.layers import CrossEntropyLoss as LdnnCE


def _loss_and_stats(criterion, out, y, stats):
    if isinstance(criterion, LdnnCE):
        return criterion(out, y, stats)
    loss = criterion(out.float(), y)
    stats[1] += (out.argmax(1) == y).sum()
    return loss


@torch.no_grad()
def validate(model, val_loader, criterion, device, *args):
    model.eval()
    dev = torch.device(device)
    stats = torch.zeros(2, dtype=torch.float32, device=dev)
    loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
    total, nb = 0, 0
    for x, y in val_loader:
        out = model(x)
        loss = _loss_and_stats(criterion, out, y, stats)
        loss_sum += loss.detach().float()
        total += y.numel()
        nb += 1
    model.train()
    if nb == 0:
        return 0.0, 0.0
    ls, correct = loss_sum.item(), stats[1].item()
    return ls / nb, 100.0 * correct / max(total, 1)


def classification_report(preds: torch.Tensor, labels: torch.Tensor, num_classes: int) -> dict:
    """precision/recall/F1 (macro, weighted, micro) from a device confusion matrix,
    matching sklearn's precision_recall_fscore_support(zero_division=0)."""
    k = num_classes
    cm = torch.bincount(labels.long() * k + preds.long(), minlength=k * k).view(k, k).double()
    tp = cm.diag()
    pred_pos = cm.sum(0)
    true_pos = cm.sum(1)
    prec = torch.where(pred_pos > 0, tp / pred_pos.clamp_min(1), torch.zeros_like(tp))
    rec = torch.where(true_pos > 0, tp / true_pos.clamp_min(1), torch.zeros_like(tp))
    f1 = torch.where(prec + rec > 0, 2 * prec * rec / (prec + rec).clamp_min(1e-300), torch.zeros_like(tp))
    support = true_pos
    present = (true_pos + pred_pos) > 0
    out = {}
    # macro: unweighted mean over labels present in y_true or y_pred (sklearn's default label set)
    n = present.sum().clamp_min(1)
    out["precision_macro"] = (prec[present].sum() / n).item()
    out["recall_macro"] = (rec[present].sum() / n).item()
    out["f1_macro"] = (f1[present].sum() / n).item()
    w = support / support.sum().clamp_min(1)
    out["precision_weighted"] = (prec * w).sum().item()
    out["recall_weighted"] = (rec * w).sum().item()
    out["f1_weighted"] = (f1 * w).sum().item()
    micro = (tp.sum() / cm.sum().clamp_min(1)).item()
    out["precision_micro"] = out["recall_micro"] = out["f1_micro"] = micro
    out["confusion_matrix"] = cm.long().cpu()
    return out


@torch.no_grad()
def evaluate(model, test_loader, criterion, device, rank=0, num_classes: int | None = None, verbose: bool = True):
    model.eval()
    dev = torch.device(device)
    stats = torch.zeros(2, dtype=torch.float32, device=dev)
    loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
    preds, labels = [], []
    nb, total = 0, 0
    for x, y in test_loader:
        out = model(x)
        loss = _loss_and_stats(criterion, out, y, stats)
        loss_sum += loss.detach().float()
        preds.append(out.argmax(1))
        labels.append(y)
        nb += 1
        total += y.numel()
    model.train()
    preds_t = torch.cat(preds) if preds else torch.zeros(0, dtype=torch.long, device=dev)
    labels_t = torch.cat(labels) if labels else torch.zeros(0, dtype=torch.long, device=dev)
    k = num_classes or int(max(int(labels_t.max().item()) + 1 if labels_t.numel() else 1, 2))
    rep = classification_report(preds_t, labels_t, k)
    loss = loss_sum.item() / max(nb, 1)
    acc = 100.0 * stats[1].item() / max(total, 1)
    if verbose:
        print(f"Rank {rank} Test Loss: {loss:.4f}, Test Accuracy: {acc:.2f}%")
        for avg in ("macro", "weighted", "micro"):
            print(f"  {avg:>8}: precision {rep['precision_' + avg]:.4f}  recall {rep['recall_' + avg]:.4f}  "
                  f"f1 {rep['f1_' + avg]:.4f}")
    evaluate.last_report = rep
    return loss, acc, preds_t.cpu().numpy(), labels_t.cpu().numpy()
