#!/usr/bin/env bash
# Launch training on every visible MI355X (one process per GPU over RCCL/xGMI).
python3 -m run.train --distributed --config_json "${1:-train_config.json}"
