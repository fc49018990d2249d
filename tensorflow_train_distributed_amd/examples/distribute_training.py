"""Flag-compatible re-implementation of the reference trainer
(/root/reference/distribute_training.py) on this framework.

    python -m tensorflow_train_distributed_amd.examples.distribute_training --job_name=ps --task_id=0
    python -m tensorflow_train_distributed_amd.examples.distribute_training --job_name=worker --task_id=0
    python -m tensorflow_train_distributed_amd.examples.distribute_training --job_name=worker --task_id=1
    (add --sync_replicas for synchronous aggregation)

Same flags/defaults as the reference (job_name, ps_hosts, worker_hosts, task_id,
sync_replicas) and the same hyper-parameters (batch 128, 2000 global steps, lr 0.01 decayed
x0.96 every int(60000/128) steps, staircase). Differences, all deliberate:
* portable paths and a stable --checkpoint_dir (Q5: relaunch resumes);
* the chief closes the token queue and shuts the PS down at the end (Q6);
* `global_step_value` is defined even if no step ran (Q9);
* --device picks cpu (default, plumbing) or gpu (HIP kernels on this rank's MI355X).
"""
from __future__ import annotations

import os
import sys
import time
from datetime import datetime

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import tensorflow_train_distributed_amd as ttd  # noqa: E402
from tensorflow_train_distributed_amd.utils import flags  # noqa: E402

BATCH_SIZE = 128
TRAINING_STEPS = 2000
MOVING_AVERAGE_DECAY = 0.99
LEARNING_RATE_DECAY_FACTOR = 0.96
INITIAL_LEARNING_RATE = 0.01
MODEL_SAVE_PATH = os.path.join(os.path.expanduser("~"), "DistributedModelSave")
DATA_PATH = os.path.join(os.path.expanduser("~"), "MNIST_Dataset")

FLAGS = flags.FLAGS
flags.DEFINE_string("job_name", "worker", ' "ps" or "worker" ')
flags.DEFINE_string("ps_hosts", "localhost:2221",
                    'Comma-separated list of hostname:port for the parameter server jobs. e.g. "tf-ps0:2221,tf-ps1:1111" ')
flags.DEFINE_string("worker_hosts", "localhost:2222,localhost:2223",
                    'Comma-separated list of hostname:port for the worker jobs. e.g. "tf-worker0:2222,tf-worker1:2223" ')
flags.DEFINE_integer("task_id", 0, "Task ID of the worker/replica running the training.")
flags.DEFINE_boolean("sync_replicas", False,
                     "Use the sync_replicas (synchronized replicas) mode, wherein the parameter updates from workers "
                     "are aggregated before applied to avoid stale gradients")
# additions (not in the reference)
flags.DEFINE_string("checkpoint_dir", "", "Checkpoint/summary dir (default: MODEL_SAVE_PATH/run-<utc>-checkpoint)")
flags.DEFINE_string("data_dir", DATA_PATH, "MNIST IDX directory (synthetic MNIST is written if missing)")
flags.DEFINE_integer("training_steps", TRAINING_STEPS, "last global step")
flags.DEFINE_integer("batch_size", BATCH_SIZE, "per-worker batch")
flags.DEFINE_integer("save_checkpoint_secs", 60, "checkpoint period (s)")
flags.DEFINE_integer("log_every", 100, "print every N local steps")
flags.DEFINE_string("device", "cpu", "cpu | gpu")
flags.DEFINE_boolean("shutdown_ps", True, "chief shuts the parameter servers down when training ends")
flags.DEFINE_integer("seed", 0, "model init / data shuffle seed")


def train(x, y_, n_workers, is_chief, device):
    global_step = ttd.train.get_or_create_global_step()
    num_batches_per_epoch = 60000 / FLAGS.batch_size
    decay_steps = int(num_batches_per_epoch)
    model = ttd.models.mnist_mlp(device=device, seed=FLAGS.seed)
    learning_rate = ttd.train.exponential_decay(INITIAL_LEARNING_RATE, global_step, decay_steps,
                                                LEARNING_RATE_DECAY_FACTOR, staircase=True)
    hook = None
    if FLAGS.sync_replicas:
        opt = ttd.train.SyncReplicasOptimizer(ttd.train.GradientDescentOptimizer(learning_rate),
                                              replicas_to_aggregate=n_workers, total_num_replicas=n_workers)
        hook = opt.make_session_run_hook(is_chief)
    else:
        opt = ttd.train.GradientDescentOptimizer(learning_rate)
    train_op = opt.minimize(model, global_step=global_step)
    loss, accuracy = train_op.loss, train_op.accuracy
    ttd.summary.scalar("loss_%d" % FLAGS.task_id, loss)
    ttd.summary.scalar("accuracy_%d" % FLAGS.task_id, accuracy)
    return global_step, loss, accuracy, train_op, hook


def main(argv=None):
    ps_hosts = FLAGS.ps_hosts.split(",")
    worker_hosts = FLAGS.worker_hosts.split(",")
    n_workers = len(worker_hosts)
    cluster = ttd.train.ClusterSpec({"ps": ps_hosts, "worker": worker_hosts})
    server = ttd.train.Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_id)
    if FLAGS.job_name == "ps":
        server.join()
        server.stop()
        return 0

    is_chief = FLAGS.task_id == 0
    mnist = ttd.data.mnist.read_data_sets(FLAGS.data_dir, seed=FLAGS.seed + FLAGS.task_id)
    device = "cpu"
    if FLAGS.device == "gpu":
        import torch
        device = "cuda:%d" % (FLAGS.task_id % max(1, torch.cuda.device_count()))
    device_setter = ttd.train.replica_device_setter(worker_device="/job:worker/task:%d" % FLAGS.task_id,
                                                    cluster=cluster)
    with ttd.device(device_setter):
        x = ttd.placeholder(np.float32, [None, 784], name="x-input")
        y_ = ttd.placeholder(np.int64, [None], name="y-input")
        global_step, loss, accuracy, train_op, sync_hook = train(x, y_, n_workers, is_chief, device)
        hooks = ([sync_hook] if sync_hook is not None else []) + \
            [ttd.train.StopAtStepHook(last_step=FLAGS.training_steps)]
        sess_config = ttd.train.ConfigProto(allow_soft_placement=True, log_device_placement=False)
        check_point_dir = FLAGS.checkpoint_dir or os.path.join(
            MODEL_SAVE_PATH, "run-%s-checkpoint" % datetime.utcnow().strftime("%Y%m%d%H%M%S"))
        global_step_value = 0
        with ttd.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief,
                                                checkpoint_dir=check_point_dir, hooks=hooks,
                                                save_checkpoint_secs=FLAGS.save_checkpoint_secs,
                                                config=sess_config) as mon_sess:
            print("session started", flush=True)
            step = 0
            start_time = time.time()
            while not mon_sess.should_stop():
                xs, ys = mnist.train.next_batch(FLAGS.batch_size)
                _, loss_value, accuracy_value, global_step_value = mon_sess.run(
                    [train_op, loss, accuracy, global_step], feed_dict={x: xs, y_: ys})
                if step > 0 and step % FLAGS.log_every == 0:
                    duration = time.time() - start_time
                    sec_per_batch = duration / max(1, global_step_value)
                    format_str = ("After %d training steps (%d global steps), loss on training batch is %g, "
                                  "accuracy is %g. (%.3f sec/batch)")
                    print(format_str % (step, global_step_value, loss_value, accuracy_value, sec_per_batch),
                          flush=True)
                step += 1
        print("total step: %d, global_step: %d" % (step, global_step_value), flush=True)
        if FLAGS.shutdown_ps:
            # coordinated shutdown (the reference's PS never exits):
            # workers report completion; the chief stops the PS tasks once all are done.
            from tensorflow_train_distributed_amd.parallel.ps import PSClient
            try:
                c = PSClient(cluster, {}, connect_timeout=10)
                done = c.counter_add("workers_done", 1)
                if is_chief:
                    deadline = time.time() + 120
                    while done < n_workers and time.time() < deadline:
                        time.sleep(0.2)
                        done = c.counter_add("workers_done", 0)
                    c.shutdown()
                c.close()
            except ttd.errors.OpError:
                pass
    return 0


if __name__ == "__main__":
    sys.exit(ttd.app.run(main))
