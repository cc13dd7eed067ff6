// render/Scene.h — the part of the reference's scene model the integrator reads
// (libs/render/include/render/Scene.h:13-227): SceneNode {id, name, type, position},
// SphereObject {radius}, and the Scene registry with its change flag. glm::vec3 is replaced by a
// three-float render::Vec3 (glm is not in this image); transforms/quaternions, unused by the
// reference integrator, are omitted.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace render
{
	struct Vec3
	{
		float x = 0.0f, y = 0.0f, z = 0.0f;
		Vec3() = default;
		Vec3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
	};

	using NodeID = uint32_t;

	enum class NodeType
	{
		SCENE_ROOT,
		SPHERE_OBJECT,
		MATERIAL,
		GROUP
	};

	class SceneNode
	{
	protected:
		static inline NodeID s_nextID = 0;  // Scene.cpp:8
		NodeID m_id;
		std::string m_name;
		NodeType m_type;
		Vec3 m_position;

	public:
		SceneNode(NodeType type, const std::string &name = "Node") : m_id(s_nextID++), m_name(name), m_type(type) {}
		virtual ~SceneNode() = default;

		NodeID GetID() const { return m_id; }
		const std::string &GetName() const { return m_name; }
		void SetName(const std::string &name) { m_name = name; }
		NodeType GetType() const { return m_type; }

		void SetPosition(const Vec3 &position) { m_position = position; }
		Vec3 GetPosition() const { return m_position; }
	};

	class SphereObject : public SceneNode
	{
	private:
		float m_radius = 1.0f;

	public:
		SphereObject(const std::string &name = "Sphere") : SceneNode(NodeType::SPHERE_OBJECT, name) {}
		float GetRadius() const { return m_radius; }
		void SetRadius(float radius) { m_radius = radius; }
	};

	class Scene
	{
	private:
		std::unique_ptr<SceneNode> m_rootNode;
		// The reference keys an unordered_map by NodeID (Scene.h:140), so its Embree geomIDs follow
		// hash-table order. An ordered map makes primitive order = creation order, deterministic on
		// every host; order only matters for exact-t ties (lowest index wins).
		std::map<NodeID, SceneNode *> m_nodeRegistry;
		std::vector<std::unique_ptr<SceneNode>> m_nodes;
		bool m_has_changes = true;

	public:
		Scene() : m_rootNode(std::make_unique<SceneNode>(NodeType::SCENE_ROOT, "Root")) {}

		SceneNode *GetRootNode() const { return m_rootNode.get(); }
		const std::map<NodeID, SceneNode *> &GetAllNodes() const { return m_nodeRegistry; }

		template <typename T, typename... Args>
		T *CreateNode(Args &&...args)
		{
			static_assert(std::is_base_of<SceneNode, T>::value, "T must be derived from SceneNode");
			auto node = std::make_unique<T>(std::forward<Args>(args)...);
			T *ptr = node.get();
			m_nodeRegistry[ptr->GetID()] = ptr;
			m_nodes.push_back(std::move(node));
			m_has_changes = true;
			return ptr;
		}

		bool hasChanges() const { return m_has_changes; }
		void markChangesProcessed() { m_has_changes = false; }
	};
} // namespace render
