"""tf.train-shaped namespace: global step, LR schedules, optimizers, sessions, hooks,
checkpoints, plus the cluster/server/placement entry points the reference calls through
tf.train (ClusterSpec, Server, replica_device_setter)."""
from .checkpoint import (Checkpoint, CheckpointManager, Saver, checkpoint_exists, get_checkpoint_state,
                         latest_checkpoint, list_variables, load_variable, update_checkpoint_state)
from .flat import FlatAdam, FlatLAMB, FlatParams, FlatSGD, ParamSpec, Schedule
from .graph import (GLOBAL_STEP, LOSSES, SUMMARIES, Fetch, GlobalStep, Placeholder, add_n, add_to_collection,
                    get_collection, get_default_graph, get_global_step, get_or_create_global_step, placeholder,
                    reset_default_graph)
from .hooks import (CheckpointSaverHook, CheckpointSaverListener, FeedFnHook, FinalOpsHook, GlobalStepWaiterHook,
                    LoggingTensorHook, NanLossDuringTrainingError, NanTensorHook, ProfilerHook, SecondOrStepTimer,
                    SessionRunArgs, SessionRunContext, SessionRunHook, SessionRunValues, StepCounterHook,
                    StopAtStepHook, SummarySaverHook, SyncReplicasOptimizerHook)
from .optimizers import (AdamOptimizer, AdamWOptimizer, GradientDescentOptimizer, LAMBOptimizer,
                         LearningRateSchedule, MomentumOptimizer, Optimizer, SyncReplicasOptimizer, TrainOp,
                         cosine_decay, exponential_decay, polynomial_decay)
from .session import (ChiefSessionCreator, ConfigProto, Coordinator, MonitoredSession, MonitoredTrainingSession,
                      Scaffold, SessionConfig, SingularMonitoredSession, WorkerSessionCreator)
from .queue_runner import QUEUE_RUNNERS, QueueRunner, SessionManager, add_queue_runner, start_queue_runners
from ..summary import FileWriterCache as SummaryWriterCache
from ..parallel.cluster import ClusterSpec
from ..parallel.ps import Server, replica_device_setter
