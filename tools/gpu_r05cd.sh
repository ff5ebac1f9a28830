#!/bin/bash
bash tools/gpu_r05c.sh && bash tools/gpu_r05d.sh
