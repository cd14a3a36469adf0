"""
Launcher (L2): let one ``ArgumentParser`` accept torchrun's flags and re-launch
the current module under ``torch.distributed.run`` when ``--distributed`` is
given.  API-compatible with the reference ``basic_utils/dist_run.py``
(reference: basic_utils/dist_run.py:13-327).

usage in a main module::

    original:   parser.parse_args(args, namespace)
    new:        parse_and_autorun(parser, args, namespace)

Differences from the reference:

* The distributed flag set is *derived from torch's own*
  ``torch.distributed.run.get_args_parser()`` at runtime instead of being a
  hand-copied subset, so the namespace handed to ``run()`` always carries every
  field the installed torch expects (fixes SURVEY C2: ``local_ranks_filter``,
  ``logs_specs``, ``numa_binding``, ... were missing on torch 2.10).
* Per-rank environment defaults for ROCm/RCCL are set before spawning
  (``OMP_NUM_THREADS`` = physical cores / GPUs as in the reference, plus
  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` which the dmabuf-only driver needs for RCCL
  IPC between ranks, and ``NCCL_IB_DISABLE=1`` for a single node).  Each worker
  pins itself to its GPU's NUMA node (``dist_util.bind_cpus_to_gpu``, in-process,
  ``DPA_NUMA_BIND``), since torchrun's ``--numa-binding`` needs ``numactl`` and
  device queries in this launcher process; the parent never initialises HIP.
"""

import os
import sys

_SKIP_DESTS = {"help", "module", "training_script", "training_script_args"}


def _gpu_count():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def run_argv_as_distributed(program_or_module, argv, dist_namespace, *, run_as_module=False):
    """Run ``torch.distributed.run`` for ``program_or_module argv...``.

    Prints the equivalent stand-alone torchrun command line first
    (reference dist_run.py:35-44).
    """
    import psutil
    from torch.distributed.run import run
    from torch.distributed.elastic.multiprocessing.errors import record

    from .dist_util import is_available
    if not is_available():
        raise RuntimeError("torch.distributed runtime not available")

    n_gpu = _gpu_count()
    os.environ.setdefault("OMP_NUM_THREADS",
                          str(max(1, (psutil.cpu_count(logical=False) or 1) // (n_gpu or 1))))
    # dmabuf IPC is the only mode the MI355X host driver supports for RCCL.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if str(getattr(dist_namespace, "nnodes", "1")) in ("1", "1:1"):
        os.environ.setdefault("NCCL_IB_DISABLE", "1")  # one node: xGMI only, no NIC probing

    if hasattr(dist_namespace, "distributed"):
        delattr(dist_namespace, "distributed")
    default = create_distributed_parser().parse_args([])
    parts = []
    for k, v in vars(dist_namespace).items():
        if not hasattr(default, k):
            continue
        if (getattr(default, k) != v and v not in ("", None)) or (k == "nproc_per_node" and str(v) != "1"):
            if isinstance(v, bool):
                if v:
                    parts.append(f"--{k}")
            else:
                parts.append(f"--{k} {v}")
    cmdline = "python3 -m torch.distributed.run " + " ".join(parts)
    cmdline += " " + "-m " * run_as_module + program_or_module + " " + " ".join(argv)
    print("[COMMANDLINE]\n" + cmdline + "\n")

    dist_namespace.module = run_as_module
    dist_namespace.training_script = program_or_module
    dist_namespace.training_script_args = list(argv)

    @record
    def main(args):
        return run(args)

    main(dist_namespace)


def create_distributed_parser(parser=None):
    """Build the torchrun-compatible flag set (+ ``--distributed``).

    The flags are copied from the installed torch's own torchrun parser, with
    ``--nproc_per_node`` defaulting to ``gpu`` when a HIP device is visible
    (reference dist_run.py:80-86).
    """
    from argparse import ArgumentParser, ArgumentDefaultsHelpFormatter, SUPPRESS
    from torch.distributed.run import get_args_parser
    import torch

    if parser is None:
        parser = ArgumentParser(add_help=False, formatter_class=ArgumentDefaultsHelpFormatter)
    parser.add_argument("--distributed", action="store_true",
                        help="run this program under torch.distributed.run")
    torch_parser = get_args_parser()
    for action in torch_parser._actions:  # noqa: SLF001 - stable argparse internals
        if action.dest in _SKIP_DESTS or not action.option_strings:
            continue
        if action.dest == "nproc_per_node":
            # device_count() does not initialise HIP in this (launcher) process: the workers
            # torchrun spawns must be the first processes to touch the GPU
            action.default = "gpu" if torch.cuda.device_count() > 0 else "1"
        if action.dest in ("no_python", "run_path"):
            action.help = SUPPRESS
        parser._add_action(action)  # noqa: SLF001
    return parser


def parse_distributed_args(parser, args=None, parse_all=True):
    """Split argv into (torchrun namespace, user args) and merge the help texts.

    Reference: basic_utils/dist_run.py:217-255.
    """
    dist_parser = create_distributed_parser()
    dist_namespace, args = dist_parser.parse_known_args(args)

    subparsers = [parser]
    try:
        if parser._subparsers is not None:  # noqa: SLF001
            from argparse import _SubParsersAction  # noqa
            sp = next(s for s in parser._subparsers._actions  # noqa: SLF001
                      if isinstance(s, _SubParsersAction))
            subparsers = list(sp._name_parser_map.values()) + [parser]  # noqa: SLF001
    except (ImportError, StopIteration):
        pass
    for _parser in subparsers:
        dist_parser.prog = " " * len(_parser.prog)
        usage = _parser._get_formatter()._format_usage(  # noqa: SLF001
            _parser.usage, _parser._actions, _parser._mutually_exclusive_groups, "")  # noqa
        _parser.usage = ("\n" if _parser is parser else "\n       ").join(usage.splitlines())
        _parser.usage += dist_parser.format_usage().replace("usage: ", " " * 7 if _parser is parser else "")
        _parser.epilog = ("NOTE - You can run this script with [torch.distributed]. "
                          "Add `--distributed` argument, and other options from "
                          "`python3 -m torch.distributed.run --help`. signature: "
                          + dist_parser.format_usage().replace("usage: ", ""))

    if parse_all:
        return dist_namespace, parser.parse_args(args)
    return dist_namespace, args


def get_main_modname():
    """Module name of the ``__main__`` frame, so we can relaunch with ``-m``.

    Reference: basic_utils/dist_run.py:258-282.
    """
    depth = 1
    try:
        while True:
            f_globals = sys._getframe(depth).f_globals  # noqa: SLF001
            if f_globals["__name__"] == "__main__":
                break
            depth += 1
    except (AttributeError, ValueError):
        return None
    spec = f_globals.get("__spec__")
    if spec is not None:
        module_name = spec.name
    elif f_globals.get("__package__") is not None and "__file__" in f_globals:
        mod = os.path.splitext(os.path.split(f_globals["__file__"])[1])[0]
        module_name = f_globals["__package__"] + "." + mod
    else:
        return None
    if module_name.endswith(".__main__"):
        module_name = module_name[:-9]
    return module_name


def parse_and_autorun(parser, args=None, namespace=None, *, module_name=None, parse_all=True):
    """Parse args; if ``--distributed`` re-run this module under torchrun and exit.

    Reference: basic_utils/dist_run.py:285-327.  In a child launched this way
    (``DIST_UTIL_AUTORUN_FLAG=1``) the dist-availability cache is forced on and
    the process title set to ``[DISTRIBUTED NODE <local_rank>]``.
    """
    if args is None:
        args = sys.argv[1:]
    dist_namespace, args = parse_distributed_args(parser, args=args, parse_all=False)

    if vars(dist_namespace).pop("distributed"):
        if module_name is None:
            module_name = get_main_modname()
        if module_name is None:
            run_as_module, program_or_module = False, sys.argv[0]
        else:
            run_as_module, program_or_module = True, module_name
        os.environ["DIST_UTIL_AUTORUN_FLAG"] = "1"
        run_argv_as_distributed(program_or_module, args, dist_namespace, run_as_module=run_as_module)
        sys.exit(0)

    if int(os.getenv("DIST_UTIL_AUTORUN_FLAG", "0")) == 1:
        from .dist_util import is_available
        is_available.cache = True
        try:
            import setproctitle  # noqa
            setproctitle.setproctitle(f"[DISTRIBUTED NODE {os.getenv('LOCAL_RANK', '0')}]")
        except ImportError:
            pass
    if parse_all:
        return parser.parse_args(args, namespace)
    return args


__all__ = ["run_argv_as_distributed", "create_distributed_parser", "parse_distributed_args",
           "get_main_modname", "parse_and_autorun"]
