"""
Entry point: ``python -m run.train [--distributed ...] --config_json cfg.json``
(reference: run/train.py:1-126, train.sh:1).

Same flow as the reference - settings -> process group -> checkpoint dir ->
logger -> seed -> data -> model -> training_args.json -> (wandb) -> TrainLoop -
with these fixes:

* Q8: the run directory name is chosen by rank 0 and broadcast, so all ranks
  agree, and an explicit ``--checkpoint_path`` enables auto-resume.
* logs append instead of truncating when resuming (Q7).
* wandb is optional (``WANDB_MODE=disabled`` or not installed -> skipped).
* the workload hooks come from the ``model`` setting (DiffuSeq / MLP diffusion
  -> ``DiffusionTrainLoop``; GPT-2 -> ``LMTrainLoop``).
"""
from torch.distributed.elastic.multiprocessing.errors import record

from config.train import TrainSettings


def create_parser():
    return TrainSettings.to_argparse(add_json=True)


def _broadcast_str(s, src=0):
    import torch.distributed as dist
    from basic_utils import dist_util
    if not dist_util.is_initialized():
        return s
    obj = [s]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


@record
def main(namespace):
    args: TrainSettings = TrainSettings.from_argparse(namespace)

    import json
    import os
    import time

    import torch

    from basic_utils import dist_util, logger
    from data import load_data_from_args
    from utils.initialization import (create_diffusion_from_config, create_model_from_config,
                                      seed_all)
    from utils.trainer import DiffusionTrainLoop, LMTrainLoop

    dist_util.setup_dist()
    rank = dist_util.get_rank()
    world = dist_util.get_world_size()
    dist_util.barrier()

    folder_name = "model_checkpoints/"
    if rank == 0:
        os.makedirs(folder_name, exist_ok=True)
    resuming = bool(args.checkpoint_path) and os.path.isdir(args.checkpoint_path)
    if not args.checkpoint_path:
        model_file = f"Run_{args.dataset}_lr{args.lr}_seed{args.seed}_{time.strftime('%Y%m%d-%H:%M:%S')}"
        args.checkpoint_path = _broadcast_str(os.path.join(folder_name, model_file))
    if rank == 0:
        os.makedirs(args.checkpoint_path, exist_ok=True)
    dist_util.barrier()

    logger.configure(dir=args.checkpoint_path,
                     format_strs=["log", "csv"] + (["stdout"] if rank == 0 else [])
                     + (["tensorboard"] if args.tensorboard and rank == 0 else []),
                     append=resuming)
    seed_all(args.seed)

    logger.log("### Creating data loader...")
    dist_util.barrier()
    common = dict(dataset=args.dataset, seq_len=args.seq_len, vocab_size=args.vocab_size,
                  seed=args.seed, model=args.model, shard=args.shard_data, rank=rank,
                  world_size=world)
    data = load_data_from_args(split='train', data_dir=args.data_dir, batch_size=args.batch_size,
                               deterministic=False, loop=True,
                               num_loader_proc=args.data_loader_workers, **common)
    data_valid = load_data_from_args(split='valid', data_dir=args.data_dir,
                                     batch_size=args.batch_size, deterministic=True, loop=True,
                                     num_loader_proc=args.data_loader_workers, **common)
    dist_util.barrier()

    logger.log("### Creating model...")
    model = create_model_from_config(**args.dict())
    model.to(dist_util.dev())
    dist_util.barrier()

    pytorch_total_params = sum(p.numel() for p in model.parameters())
    logger.log(f'### The parameter count is {pytorch_total_params}')

    training_args_path = f'{args.checkpoint_path}/training_args.json'
    if not os.path.exists(training_args_path):
        logger.log(f'### Saving the hyperparameters to {training_args_path}')
        if rank == 0:
            with open(training_args_path, 'w') as fp:
                json.dump(args.dict(), fp, indent=2)

    if rank == 0 and os.getenv("WANDB_MODE", "disabled") != "disabled":
        try:
            import wandb
            wandb.init(mode=os.getenv("WANDB_MODE"))
            wandb.config.update(args.dict(), allow_val_change=True)
        except ImportError:
            logger.log("wandb not installed; skipping")
    dist_util.barrier()

    logger.log("### Training...")
    kwargs = dict(
        model=model, data=data, batch_size=args.batch_size, microbatch=args.microbatch, lr=args.lr,
        ema_rate=args.ema_rate, log_interval=args.log_interval, save_interval=args.save_interval,
        resume_checkpoint=args.resume_checkpoint, weight_decay=args.weight_decay,
        learning_steps=args.learning_steps, checkpoint_path=args.checkpoint_path,
        gradient_clipping=args.gradient_clipping, eval_data=data_valid,
        eval_interval=args.eval_interval, eval_callbacks=[],
        ddp_engine=args.ddp_engine, precision=args.precision, bucket_cap_mb=args.ddp_bucket_cap_mb,
        first_bucket_mb=args.ddp_first_bucket_mb, grad_reduce_dtype=args.grad_reduce_dtype,
        shard_optimizer=args.shard_optimizer,
        exec_microbatch=args.exec_microbatch,
        overlap_microbatches=args.overlap_microbatches, defer_wgrad=args.defer_wgrad,
        log_cross_rank_mean=args.log_cross_rank_mean, nan_guard=args.nan_guard,
        debug_anomaly=args.debug_anomaly, consistency_check_interval=args.consistency_check_interval,
        profile_steps=args.profile_steps, roctx=args.roctx, save_rng_state=args.save_rng_state)
    if args.model == "gpt2":
        loop = LMTrainLoop(**kwargs)
    else:
        diffusion, sampler = create_diffusion_from_config(**args.dict())
        loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, **kwargs)
    loop.run_loop()
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        dist_util.barrier()


if __name__ == "__main__":
    from basic_utils.dist_run import parse_and_autorun
    main(parse_and_autorun(create_parser()))
