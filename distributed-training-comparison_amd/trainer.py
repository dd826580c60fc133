"""Trainer and CLI mirroring the reference's src/single and src/ddp entry points.

Same flags (src/ddp/config.py:4-39; src/single/config.py differs only in ckpt-path/epoch
defaults), same flow (main.py -> Trainer.fit -> _train_epoch -> validate -> checkpoint -> test),
same step (single/trainer.py:131-147, ddp/trainer.py:149-167 incl. the per-step dist.barrier()),
on the native modules. Differences, all forced by this environment and documented in DESIGN.md:
CIFAR-100 is replaced by a seeded synthetic stand-in (no download), TensorBoard scalars go to
``scalars.jsonl`` (tensorboardX is not installed), and the model always computes in bf16.
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
from typing import Tuple

import torch
import torch.distributed as dist

from . import data as D
from .amp import GradScaler, autocast
from .nn import CrossEntropyLoss, ResNet18, SyncBatchNorm
from .optim import SGD
from .parallel import DDP, DataParallel, barrier


def load_config(argv=None, mode: str = "ddp"):
    p = argparse.ArgumentParser()
    p.add_argument("--dset", type=str, default="cifar100")
    p.add_argument("--dpath", type=str, default="data/")
    p.add_argument("--ckpt-path", type=str, default=f"src/{mode}/checkpoints/")
    p.add_argument("--seed", type=int, default=42, help="Seed for reproducibility")
    p.add_argument("--workers", type=int, default=4)
    p.add_argument("--eval-step", type=int, default=300)
    p.add_argument("--amp", action="store_true", default=False, help="PyTorch(>=1.6.x) AMP")
    p.add_argument("--contain-test", action="store_true", default=False)
    if mode == "ddp":
        p.add_argument("--world-size", type=int, default=1, help="Total number of processes to run")
        p.add_argument("--rank", type=int, default=0)
        p.add_argument("--dist-backend", type=str, default="nccl")
        p.add_argument("--dist-url", default="tcp://127.0.0.1:3456", type=str)
        p.add_argument("--sync-bn", action="store_true", default=False,
                       help="SyncBatchNorm.convert_sync_batchnorm (README.md:40; off in the reference)")
    p.add_argument("--epoch", type=int, default=200 if mode == "single" else 100)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--model", type=str, default="resnet18")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--weight-decay", type=float, default=0.0001)
    p.add_argument("--lr-decay-step-size", type=int, default=60)
    p.add_argument("--lr-decay-gamma", type=float, default=0.1)
    # synthetic-data size knobs (not in the reference: CIFAR-100 cannot be downloaded here)
    p.add_argument("--synthetic-train", type=int, default=50000)
    p.add_argument("--synthetic-test", type=int, default=10000)
    p.add_argument("--max-steps", type=int, default=0, help="stop each epoch after N steps (0 = full epoch)")
    p.add_argument("--device-data", action="store_true", default=False,
                   help="HBM-resident uint8 dataset + on-GPU crop/flip/normalize (data.DeviceLoader)")
    if mode == "dp":  # not in the reference (nn.DataParallel takes every visible GPU): replica placement
        p.add_argument("--device-ids", type=lambda v: [int(d) for d in v.split(",")], default=None,
                       help="comma-separated GPU ids of the replicas (may repeat); default: all visible")
    return p.parse_args(argv)


def accuracy(output, target, topk=(1,)):
    """utils.py:18-31."""
    maxk = max(topk)
    batch_size = target.size(0)
    _, pred = output.topk(maxk, 1, True, True)
    pred = pred.t()
    correct = pred.eq(target.reshape(1, -1).expand_as(pred))
    return [correct[:k].reshape(-1).float().sum(0).mul_(100.0 / batch_size) for k in topk]


class AverageMeter:
    """utils.py:34-48."""

    def __init__(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, val: float, n: int = 1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class Trainer:
    def __init__(self, hparams, model, scaler, rank: int = 0, ngpus_per_node: int = 1, distributed: bool = False,
                 data_parallel: bool = False):
        self.hparams = hparams
        self.rank = rank
        self.distributed = distributed
        self.data_parallel = data_parallel
        self.device = torch.device("cuda", rank if distributed else torch.cuda.current_device())
        self.model = model.to(self.device)
        if data_parallel:
            self.model = DataParallel(self.model, device_ids=getattr(hparams, "device_ids", None))  # dp/trainer.py:27
        if distributed:
            self.model = DDP(self.model, device_ids=[rank], find_unused_parameters=True)   # ddp/trainer.py:31
            hparams.batch_size = int(hparams.batch_size / ngpus_per_node)                  # ddp/trainer.py:34
        self.scaler = scaler
        self.optimizer, self.lr_scheduler = self.configure_optimizers()
        self.criterion = CrossEntropyLoss()
        if getattr(hparams, "device_data", False):
            self._device_loaders(hparams, distributed)
        else:
            ds = D.SyntheticCIFAR100(n=hparams.synthetic_train)
            self.train_loader, self.train_sampler, self.val_loader = D.get_trn_val_loader(
                batch_size=hparams.batch_size, valid_size=0.1, num_workers=hparams.workers, pin_memory=True,
                distributed=distributed, dataset=ds)
            self.test_loader = D.get_tst_loader(batch_size=hparams.batch_size, num_workers=1, pin_memory=True,
                                                distributed=distributed, n=hparams.synthetic_test)
        self.global_step = 0
        self.global_top1_acc = 0.0
        self.eval_step = hparams.eval_step
        self.version = None
        if rank == 0:
            self.version = 0
            while True:
                self.save_path = os.path.join(hparams.ckpt_path, f"version-{self.version}")
                if not os.path.exists(self.save_path):
                    os.makedirs(self.save_path)
                    break
                self.version += 1
            logging.basicConfig(filename=os.path.join(self.save_path, "experiment.log"), level=logging.INFO,
                                format="%(asctime)s > %(message)s", force=True)
            with open(os.path.join(self.save_path, "hparams.json"), "w") as f:
                json.dump(vars(hparams), f, indent=1)
            self._scalars = open(os.path.join(self.save_path, "scalars.jsonl"), "a")

    def _device_loaders(self, hparams, distributed):
        """--device-data: the loaders of dataset.py:15-168 with the transforms on the GPU
        (D.DeviceLoader over HBM-resident uint8 CIFAR-shaped data): same 45k/5k split, the same
        DistributedSampler (DDP) or per-epoch random order (single/dp), drop_last on train, train
        transform with crop+flip, valid without, test normalized with the ImageNet statistics of
        dataset.py:139-142 and sharded by a DistributedSampler under DDP (dataset.py:158)."""
        imgs, tg = D.synthetic_cifar_u8(n=hparams.synthetic_train, seed=hparams.seed)
        train_idx, valid_idx = D.train_valid_split(len(tg), 0.1, True)
        sampler = (D.DistributedSampler(train_idx) if distributed
                   else torch.utils.data.SubsetRandomSampler(list(range(len(train_idx)))))
        bs = hparams.batch_size
        self.train_loader = D.DeviceLoader(imgs, tg, bs, subset_idx=train_idx, sampler=sampler, train=True,
                                           seed=hparams.seed, device=self.device)
        self.train_sampler = self.train_loader
        self.val_loader = D.DeviceLoader(imgs, tg, bs, subset_idx=valid_idx, train=False, drop_last=False,
                                         device=self.device)
        timgs, ttg = D.synthetic_cifar_u8(n=hparams.synthetic_test, seed=hparams.seed + 1)
        # DistributedSampler(test_dataset) with its default shuffle=True, exactly dataset.py:158: rank 0
        # tests the same (shuffled) 1/W subset the reference's rank 0 does
        tsampler = D.DistributedSampler(range(len(ttg))) if distributed else None
        self.test_loader = D.DeviceLoader(timgs, ttg, bs, sampler=tsampler, train=False, drop_last=False,
                                          mean=D.IMAGENET_MEAN, std=D.IMAGENET_STD, device=self.device)

    def _log_scalar(self, tag, values, step):
        if self.rank == 0:
            self._scalars.write(json.dumps({"tag": tag, "step": step, **values}) + "\n")
            self._scalars.flush()

    def configure_optimizers(self):
        optimizer = SGD(self.model.parameters(), lr=self.hparams.lr, weight_decay=self.hparams.weight_decay,
                        momentum=0.9, nesterov=True)                                      # trainer.py:92-98
        scheduler = torch.optim.lr_scheduler.StepLR(optimizer, step_size=self.hparams.lr_decay_step_size,
                                                    gamma=self.hparams.lr_decay_gamma)    # trainer.py:101-105
        return optimizer, scheduler

    def save_checkpoint(self, epoch: int, val_acc: float, model) -> None:
        logging.info(f"Val acc increased ({self.global_top1_acc:.4f} -> {val_acc:.4f}). Saving model ...")
        new_path = os.path.join(self.save_path, f"best_model_epoch_{epoch}_acc_{val_acc:.4f}.pt")
        for filename in glob.glob(os.path.join(self.save_path, "*.pt")):
            os.remove(filename)
        torch.save({k: v.contiguous() for k, v in model.state_dict().items()}, new_path)
        self.global_top1_acc = val_acc

    def fit(self):
        for epoch in range(self.hparams.epoch):
            if self.distributed or isinstance(self.train_loader, D.DeviceLoader):
                self.train_sampler.set_epoch(epoch)                                       # trainer.py:125
            logging.info(f"* Learning Rate: {self.optimizer.param_groups[0]['lr']:.5f}")
            result = self._train_epoch(epoch)
            if self.rank == 0 and result["val_acc"] > self.global_top1_acc:
                self.save_checkpoint(epoch, result["val_acc"], self.model)
            self.lr_scheduler.step()
        return self.version

    def _train_epoch(self, epoch: int) -> dict:
        train_loss = AverageMeter()
        self.model.train()
        for step, (img, label) in enumerate(self.train_loader):
            if self.hparams.max_steps and step >= self.hparams.max_steps:
                break
            img = img.to(self.device, non_blocking=True)
            label = label.to(self.device, non_blocking=True)
            self.optimizer.zero_grad()
            if self.hparams.amp:
                with autocast():
                    logit = self.model(img)
                    loss = self.criterion(logit, label)
                if self.distributed:
                    barrier()  # dist.barrier() on the native communicator            # trainer.py:156
                self.scaler.scale(loss).backward()
                self.scaler.step(self.optimizer)
                self.scaler.update()
            else:
                logit = self.model(img)
                loss = self.criterion(logit, label)
                if self.distributed:
                    barrier()                                                             # trainer.py:163
                loss.backward()
                self.optimizer.step()
            train_loss.update(loss.item())
            self.global_step += 1
            if self.rank == 0 and self.global_step % self.eval_step == 0:
                tag = "DDP" if self.distributed else ("DP" if self.data_parallel else "Single")
                logging.info(f"[{tag} Version {self.version} Epoch {epoch}] "
                             f"global step: {self.global_step}, train loss: {loss.item():.3f}")
        result = {"val_loss": 0.0, "val_acc": 0.0, "train_loss": train_loss.avg}
        if self.rank == 0:
            val_loss, val_acc = self.validate(epoch)
            self._log_scalar("lr", {"lr": self.optimizer.param_groups[0]["lr"]}, epoch)
            self._log_scalar("loss/epoch", {"val": val_loss, "train": train_loss.avg}, epoch)
            self._log_scalar("acc/epoch", {"val": val_acc}, epoch)
            logging.info(f"** global step: {self.global_step}, val loss: {val_loss:.3f}, val_acc: {val_acc:.2f}%")
            result.update(val_loss=val_loss, val_acc=val_acc)
        return result

    def _module(self):
        # DDP: rank 0 evaluates the unwrapped module; DP evaluates through the replicas
        # (dp/trainer.py:121-129 calls self.model, the DataParallel wrapper)
        return self.model.module if self.distributed else self.model

    def validate(self, epoch: int) -> Tuple[float, float]:
        val_loss, top1 = AverageMeter(), AverageMeter()
        net = self._module()  # rank 0 evaluates the unwrapped module
        net.eval()
        with torch.no_grad():
            for img, label in self.val_loader:
                img, label = img.to(self.device), label.to(self.device)
                pred = net(img)
                val_loss.update(self.criterion(pred, label).item())
                top1.update(accuracy(pred, label, topk=(1,))[0].item())
        net.train()
        return val_loss.avg, top1.avg

    def test(self, state_dict) -> dict:
        test_loss, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter()
        self.model.load_state_dict(state_dict)
        net = self._module()
        net.eval()
        with torch.no_grad():
            for img, label in self.test_loader:
                img, label = img.to(self.device), label.to(self.device)
                pred = net(img)
                test_loss.update(self.criterion(pred, label).item())
                p1, p5 = accuracy(pred, label, topk=(1, 5))
                top1.update(p1.item())
                top5.update(p5.item())
        logging.info(f"** Test Loss: {test_loss.avg:.4f}")
        logging.info(f"** Top-1 Accuracy: {top1.avg:.4f}%")
        logging.info(f"** Top-5 Accuracy: {top5.avg:.4f}%")
        return {"test_loss": test_loss.avg, "top_1_acc": top1.avg, "top_5_acc": top5.avg}


def _run(hparams, rank, ngpus, distributed, data_parallel=False):
    D.fix_seed(hparams.seed)
    scaler = GradScaler() if hparams.amp else None
    model = ResNet18()
    if getattr(hparams, "sync_bn", False):
        model = SyncBatchNorm.convert_sync_batchnorm(model)
    trainer = Trainer(hparams, model, scaler, rank, ngpus, distributed, data_parallel)
    version = trainer.fit()
    if rank == 0 and hparams.contain_test:
        path = glob.glob(os.path.join(hparams.ckpt_path, f"version-{version}/best_model_*.pt"))
        if path:
            state = torch.load(path[0], weights_only=True)
            print(json.dumps(trainer.test(state)))
    return trainer


def main_worker(rank, ngpus_per_node, hparams):
    """ddp/main.py:14-39."""
    hparams.rank = hparams.rank * ngpus_per_node + rank
    torch.cuda.set_device(rank)
    dist.init_process_group(backend=hparams.dist_backend, init_method=hparams.dist_url,
                            world_size=hparams.world_size, rank=hparams.rank)
    try:
        _run(hparams, rank, ngpus_per_node, True)
    finally:
        dist.destroy_process_group()


def main(argv=None, mode: str = "ddp"):
    hparams = load_config(argv, mode)
    if mode == "single":
        return _run(hparams, 0, 1, False)
    if mode == "dp":  # src/dp/main.py: one process, nn.DataParallel over every visible GPU
        return _run(hparams, 0, torch.cuda.device_count(), False, data_parallel=True)
    if mode != "ddp":
        raise ValueError(f"unknown mode {mode!r} (single, dp, ddp)")
    import torch.multiprocessing as mp

    ngpus_per_node = torch.cuda.device_count()
    hparams.world_size = ngpus_per_node * hparams.world_size
    mp.spawn(main_worker, nprocs=ngpus_per_node, args=(ngpus_per_node, hparams))
