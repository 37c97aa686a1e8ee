# the val and training-step profiles at this commit (the training step on 16,384 rays: the same full chunks)
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/profile.sh r02k_val --mode val --steps 3 --warmup 1 && bash scripts/profile.sh r02k_train_step --mode train_step --rays 16384 --steps 2 --warmup 1
echo rc=$?
