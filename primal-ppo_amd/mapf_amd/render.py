"""Evaluation GIFs (driver.py:232-286): frames from the device renderer and util.make_gif.

The frames come from `BatchedMapfGym.render` / `MapfGym._render` (the HIP kernel behind
`mapf_render`, renderWorld util.py:189-232); this module only encodes them.  The reference
writes GIFs with imageio (util.py:304-308), absent from this image: Pillow writes the same
animated GIF (palette images, one frame per step, looping) -- `subrectangles=True` there is a
size optimisation of the encoding, not of the pictures.
"""
import numpy as np


def make_gif(images, file_name, duration_ms=100):
    """util.make_gif: write the uint8 RGB frames `images` ([T, H, W, 3] array or a list of them)
    to an animated GIF at `file_name`."""
    from PIL import Image
    frames = [Image.fromarray(np.ascontiguousarray(np.asarray(im, dtype=np.uint8))) for im in images]
    if not frames:
        raise ValueError("make_gif: no frames")
    print("writing gif to ", file_name)
    frames[0].save(file_name, save_all=True, append_images=frames[1:], duration=duration_ms, loop=0,
                   optimize=True)
    print("wrote gif")


def episode_frames(env, steps, policy=None, env_index=0, scale=20):
    """Frames of one env of a BatchedMapfGym over `steps` committed steps (driver.py's
    evaluate loop appends env._render() before the first step and after each): the given
    policy (actions int32 [B, N] on the device) or the uniform random one."""
    frames = [env.render([env_index], scale=scale)[0].cpu().numpy()]
    for _ in range(steps):
        acts = env.random_actions() if policy is None else policy(env)
        env.step(acts)
        frames.append(env.render([env_index], scale=scale)[0].cpu().numpy())
    return np.stack(frames)
