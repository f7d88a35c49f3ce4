#!/bin/bash
set -e
tools/gpu_r04c.sh r04g
tools/gpu_pmc_calib.sh
