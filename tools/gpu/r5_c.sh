#!/bin/bash
bash tools/gpu/r5_ab.sh bp lib_bp && bash tools/gpu/r5_prof.sh r5c
