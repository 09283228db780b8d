"""ORACLE (test infrastructure only — imported by tests/, never by the product path).

CPU restatement of the reference's eval-time KRRNLoss terms with the same torch ops:
MapLoss + l1 / cosine / cross_entropy (lib/network/loss_utils.py:8-70) and PoseLoss
(lib/network/loss.py:19-42). The KeOps argkmin (train.py:126, pykeops absent here) is restated
as a brute-force argmin of the squared distance (ties -> lower index: torch.argmin's rule).
"""
import torch
import torch.nn as nn


def cosine(x, tgt):  # loss_utils.py:8-10
    return 1.0 - nn.CosineSimilarity(dim=1, eps=1e-6)(x, tgt)


def l1(x, tgt):  # loss_utils.py:12-13
    return torch.abs(x - tgt).sum(dim=1)


def cross_entropy(x, tgt, eps=1e-6):  # loss_utils.py:15-17
    x = -torch.log(torch.softmax(x, 1) + torch.tensor(eps))
    return torch.gather(x, 1, tgt).squeeze(1)


def map_loss(fn, x, target):  # MapLoss.forward, loss_utils.py:55-70 ('elementwise_mean')
    loss = fn(x, target)
    invalid = torch.all(target == 0., dim=1)
    loss[invalid] = 0.0
    return loss.sum() / (~invalid).sum().double()


def knn_nearest(query, cand):
    d = ((query[:, None, :] - cand[None, :, :]) ** 2).sum(-1)
    return torch.argmin(d, dim=1)


def pose_loss(pred_r, pred_t, targets, model_points, idxs, sym_list):  # loss.py:26-42
    pred_points = model_points @ pred_r.permute(0, 2, 1) + pred_t
    tgts = []
    for b in range(pred_points.size(0)):
        tgt = targets[b]
        if int(idxs[b]) in sym_list:
            tgt = torch.index_select(tgt, 0, knn_nearest(pred_points[b], tgt).view(-1))
        tgts.append(tgt)
    return torch.mean(torch.norm(pred_points - torch.stack(tgts, 0), dim=2), dim=1).mean()


def krrn_loss(pred, gt, sym_list, opt_pose=True):  # KRRNLoss.forward without the weights
    out = {
        "loss_xyz": map_loss(l1, pred["xyz"], gt["xyz"]),
        "loss_normal": map_loss(cosine, pred["normal"], gt["normal"]),
        "loss_region": map_loss(cross_entropy, pred["region"], gt["region"].unsqueeze(1).long()),
        "loss_mask": map_loss(cross_entropy, pred["mask"], gt["multi_cls_mask"].unsqueeze(1).long()),
    }
    if opt_pose:
        out["loss_add"] = pose_loss(gt["target_r"], pred["pred_t"].unsqueeze(1), gt["target"], gt["model_points"],
                                    gt["cls_id"].view(-1), sym_list)
    return out
