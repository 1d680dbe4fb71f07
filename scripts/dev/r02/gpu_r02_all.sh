bash scripts/gpu_r02_tests.sh && bash scripts/gpu_r02_profiles.sh
