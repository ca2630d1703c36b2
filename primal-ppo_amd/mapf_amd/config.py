"""Configuration mirror of the reference's alg_parameters.py.

The class names and attribute names follow alg_parameters.py (EnvParameters
:27-48, TrainingParameters :50-78, NetParameters :100-105) so reference code
reading them keeps working; `make_config` turns them into the C struct
mapf_config (include/mapf.h).
"""
import ctypes


class EnvParameters:
    N_AGENTS = 2
    N_ACTIONS = 5
    EPISODE_LEN = 256
    FOV_SIZE = 9
    FOV_Heuristic = 5
    WORLD_SIZE = (10, 40)
    OBSTACLE_PROB = (0.0, 0.3)
    ACTION_COST = -0.3
    IDLE_COST = -0.3
    GOAL_REWARD = 1.5
    COLLISION_COST = -2
    HUMAN_COLLISION_COST = -2
    REPEAT_POS = -0.35
    BLOCKING_COST = 0
    PENALTY_RADIUS = 5
    CONSTRAINT_VIOLATION_COST = -1.0
    LIFELONG = True


class TrainingParameters:
    lr = 1e-5
    GAMMA = 0.95
    LAM = 0.95
    CLIP_RANGE = 0.2
    MAX_GRAD_NORM = 10
    ENTROPY_COEF = 0.01
    VALUE_COEF = 0.08
    POLICY_COEF = 10
    VALID_COEF = 0.5
    BLOCK_COEF = 0.5
    COST_VALUE_COEF = 0.0
    COST_COEF = 0.0
    COST_LIMIT_PER_AGENT = 5
    N_EPOCHS = 10
    N_ENVS = 16
    N_MAX_STEPS = 3e7
    N_STEPS = 2 ** 8
    MINIBATCH_SIZE = int(2 ** 8)
    DEMONSTRATION_PROB = 0
    USE_INFLATED_HUMAN = True
    USE_HUMAN_TRAJECTORY_PREDICTION = True
    K_TIMESTEP_PREDICT = 5
    MINUS_ADV_WITH_CADV = True


class NetParameters:
    NET_SIZE = 512
    NUM_CHANNEL = 5 + int(TrainingParameters.USE_HUMAN_TRAJECTORY_PREDICTION)
    GOAL_REPR_SIZE = 12
    VECTOR_LEN = 4


class LagrangianParameters:
    LAGRANGIAN_TYPE = 0
    INIT_VALUE = 1.0
    UPPER_BOUND = 20.0
    LR = 5e-2
    KP = 0.1
    KI = 0.01
    KD = 0.01
    COST_MOVING_AVG_ALPHA = 0.95
    DELTA_MOVING_AVG_ALPHA = 0.95


class SetupParameters:
    SEED = 1234
    USE_GPU_LOCAL = True
    USE_GPU_GLOBAL = True
    NUM_GPU = 1


class MapfConfig(ctypes.Structure):
    """include/mapf.h: mapf_config (field for field)."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "num_envs", "num_agents", "height", "width", "fov", "num_channel",
        "use_da", "use_hp", "lifelong", "human_mode", "goal_mode", "fix_choice",
        "shared_map", "keep_bfs", "max_seq", "max_human_seq", "k_predict", "penalty_radius")] + \
        [(n, ctypes.c_float) for n in ("action_cost", "collision_cost", "human_collision_cost",
                                       "repeat_cost", "goal_reward")] + \
        [("env_offset", ctypes.c_int32), ("reserved", ctypes.c_uint32), ("seed", ctypes.c_uint64)]


HUMAN_MODES = {"looping": 0, "random": 1, "fixed_path": 2}
GOAL_MODES = {"sequence": 0, "random": 1}


def make_config(num_envs, height, width, *, num_agents=None, fov=None, num_channel=None, use_da=False,
                use_hp=False, human_mode="random", goal_mode="random", fix_choice=1, shared_map=True,
                keep_bfs=True, max_seq=1, max_human_seq=2, env_offset=0, seed=None):
    """Build a mapf_config from the reference's parameter classes."""
    c = MapfConfig()
    c.num_envs = num_envs
    c.num_agents = EnvParameters.N_AGENTS if num_agents is None else num_agents
    c.height, c.width = height, width
    c.fov = EnvParameters.FOV_SIZE if fov is None else fov
    c.num_channel = NetParameters.NUM_CHANNEL if num_channel is None else num_channel
    c.use_da, c.use_hp = int(use_da), int(use_hp)
    c.lifelong = int(EnvParameters.LIFELONG)
    c.human_mode = HUMAN_MODES[human_mode] if isinstance(human_mode, str) else int(human_mode)
    c.goal_mode = GOAL_MODES[goal_mode] if isinstance(goal_mode, str) else int(goal_mode)
    c.fix_choice = int(fix_choice)
    c.shared_map = int(shared_map)
    c.keep_bfs = int(keep_bfs)
    c.max_seq = max_seq
    c.max_human_seq = max_human_seq
    c.k_predict = TrainingParameters.K_TIMESTEP_PREDICT
    c.penalty_radius = EnvParameters.PENALTY_RADIUS
    c.action_cost = EnvParameters.ACTION_COST
    c.collision_cost = EnvParameters.COLLISION_COST
    c.human_collision_cost = EnvParameters.HUMAN_COLLISION_COST
    c.repeat_cost = EnvParameters.REPEAT_POS
    c.goal_reward = EnvParameters.GOAL_REWARD
    c.env_offset = env_offset
    c.seed = SetupParameters.SEED if seed is None else seed
    return c
