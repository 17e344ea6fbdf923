#!/bin/bash
bash tools/gpu/r5_e.sh && bash tools/gpu/r5_f.sh
